"""Summarise wait-state / instruction-mix PMC passes of one trace_kernel frame into <dst>/waits.json.

Inputs: rocprofv3 --pmc pass directories (tools/gpu.sh `pmc:` steps, each one bench frame: --steps 1
--warmup 0) whose bench run printed its JSON line to <pass dir>.log.  Counters of the trace_kernel
dispatches are summed per pass; SQ_WAVE_CYCLES (in every pass) normalises each pass's cycle counters.

  issue share       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES    (a wave issuing)
  dependency wait   = SQ_WAIT_ANY / SQ_WAVE_CYCLES           (parked on s_waitcnt / barrier)
  issue-slot wait   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES      (ready, but the SIMD's pipe is taken)
  (the three are disjoint and sum to ~1: MI355X_MICROARCH.md, SQ counters)
  LDS issue stall   = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES      (a sub-bucket of the issue-slot wait)
  per segment       = SQ_INSTS_* / segments of the frame
  spill stores      ~ SQ_INSTS_VMEM_WR - 3 x units published (the partial sums' three f64 stores)

usage: python tools/pmc_waits.py <profiles/TAG> <pass_dir> [<pass_dir> ...]
"""
import csv
import glob
import json
import os
import sys


def summed(pass_dir):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"]]
    agg = {}
    for r in rows:
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return f, rows, agg


def bench_line(pass_dir):
    for line in open(pass_dir.rstrip("/") + ".log"):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {pass_dir}.log")


def main(dst, *passes):
    os.makedirs(dst, exist_ok=True)
    out, sources, frame = {}, [], None
    for i, p in enumerate(passes):
        f, rows, agg = summed(p)
        name = os.path.join(dst, f"pmc_waits_pass{i + 1}.csv")
        with open(name, "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        b = bench_line(p)
        seg = b["roofline"]["segments_per_launch"] * b["roofline"].get("launches_per_step", 1)
        units = b["config"]["width"] * b["config"]["height"] * b["config"]["n_chunks"]
        frame = frame or {"workload": b["config"]["workload"], "segments": seg, "units": units}
        wc = agg.get("SQ_WAVE_CYCLES")
        for k, v in agg.items():
            if k == "SQ_WAVE_CYCLES":
                continue
            if k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) and wc:
                out[k + "/SQ_WAVE_CYCLES"] = round(v / wc, 4)
            elif k.startswith("SQ_INSTS") or k == "SQ_LDS_BANK_CONFLICT":
                out[k + "/segment"] = round(v / seg, 3)
            out.setdefault("raw", {})[k] = v
        sources.append(os.path.basename(name))
    if "SQ_INSTS_VMEM_WR" in out.get("raw", {}):
        out["spill_store_insts/segment (VMEM_WR - 3 x units)"] = round(
            (out["raw"]["SQ_INSTS_VMEM_WR"] - 3.0 * frame["units"]) / frame["segments"], 4)
    res = {**frame, **out, "source": f"{dst}: " + ", ".join(sources)}
    json.dump(res, open(os.path.join(dst, "waits.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "raw"}))


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
