"""Summarise the VALU PMC passes of one trace_kernel dispatch into profiles/valu.json (read by bench.py).

Inputs: rocprofv3 --pmc pass directories (tools/gpu.sh `pmc:` steps) whose bench run printed its JSON line
to <pass dir>.log.  Each pass profiles ONE frame (bench --steps 1 --warmup 0): the trace_kernel dispatches
of that frame (one per sample pass) are summed, and every pass sees the same deterministic workload
(same seed -> same segments).

  busy_frac   = SQ_ACTIVE_INST_VALU / (SQ_WAVE_CYCLES / waves_per_simd)   (SIMD issue slots used by VALU)
  lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)        (active lanes per VALU cycle)
  f64 FLOPs   = (ADD_F64 + MUL_F64 + 2 FMA_F64) wave-instructions x 64 x lane_util

usage: python tools/pmc_valu.py <profiles/TAG> <waves_per_simd> <pass_dir> [<pass_dir> ...]
(PMC_NO_TOP=1: write <profiles/TAG>/valu.json only, not the top-level copy bench.py reads)
"""
import csv
import glob
import json
import os
import sys


def dispatch_counters(pass_dir):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"]]
    ids = sorted({r["Dispatch_Id"] for r in rows}, key=int)
    agg = {}
    for r in rows:
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return f, rows, agg, ids


def bench_line(pass_dir):
    for line in open(pass_dir.rstrip("/") + ".log"):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {pass_dir}.log")


def main(dst, waves_per_simd, *passes):
    os.makedirs(dst, exist_ok=True)
    c, sources, segs, cfg = {}, [], set(), None
    for i, p in enumerate(passes):
        f, rows, agg, did = dispatch_counters(p)
        c.update(agg)
        out = os.path.join(dst, f"pmc_valu_pass{i + 1}.csv")
        with open(out, "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        b = bench_line(p)
        assert len(did) == b["roofline"].get("launches_per_step", 1), f"{p}: dispatches {did} vs the frame's launches"
        segs.add(b["roofline"]["segments_per_launch"] * b["roofline"].get("launches_per_step", 1))
        cfg = b["config"]
        sources.append(f"{os.path.basename(out)} (dispatches {','.join(did)})")
    assert len(segs) == 1, f"passes saw different workloads: {segs}"
    seg = segs.pop()
    wps = float(waves_per_simd)
    lane = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    f64_insts = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2.0 * c["SQ_INSTS_VALU_FMA_F64"]
    v = {
        "scene": cfg["scene"], "bvh": cfg["bvh"], "size": [cfg["width"], cfg["height"]], "spp": cfg["spp"],
        "segments": seg, "waves_per_simd": wps,
        "valu_busy_frac": round(c["SQ_ACTIVE_INST_VALU"] / (c["SQ_WAVE_CYCLES"] / wps), 4),
        "lane_util": round(lane, 4),
        "valu_insts_per_segment": round(c["SQ_INSTS_VALU"] / seg, 3),
        "salu_insts_per_segment": round(c.get("SQ_INSTS_SALU", 0.0) / seg, 3),
        "f64_flops_per_segment": round(f64_insts * 64.0 * lane / seg, 3),
        "f64_share_of_valu": round((c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                                    c["SQ_INSTS_VALU_FMA_F64"]) / c["SQ_INSTS_VALU"], 4),
        "counters": c,
        "source": f"{dst}: " + ", ".join(sources),
    }
    json.dump(v, open(os.path.join(dst, "valu.json"), "w"), indent=1)
    if not os.environ.get("PMC_NO_TOP"):  # (a config other than the headline: keep profiles/valu.json)
        json.dump(v, open(os.path.join(os.path.dirname(dst.rstrip("/")), "valu.json"), "w"), indent=1)
    print(json.dumps({k: v[k] for k in v if k != "counters"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *sys.argv[3:])
