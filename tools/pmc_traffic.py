"""Summarise a `tools/gpu.sh <tag> prof pmc:FETCH_SIZE pmc:WRITE_SIZE` run: kernel-trace stats + the mean
per-dispatch HBM traffic of the trace kernel from the FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md §HBM prescribes (counters in KiB; gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced reads -> x2).  A frame runs one trace launch per sample pass: the figures are per launch, like
bench.py's roofline.  Writes profiles/<round>/ (copied CSV summaries) and profiles/traffic.json (read by
bench.py).

usage: python tools/pmc_traffic.py <gpurun_out/TAG> <profiles/ROUND> <workload> <bvh>
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys


def per_dispatch(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return vals


def main(src, dst, workload, bvh):
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "prof", "**", "*kernel_stats.csv"), recursive=True) + \
            glob.glob(os.path.join(src, "prof", "**", "*domain_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, os.path.basename(f).replace("run_", "")))
    def pass_csv(name):
        return glob.glob(os.path.join(src, f"pmc_{name}", "**", "*counter_collection.csv"), recursive=True)[0]
    fetch = per_dispatch(pass_csv("FETCH_SIZE"), "trace_kernel")
    write = per_dispatch(pass_csv("WRITE_SIZE"), "trace_kernel")
    for name in ("FETCH_SIZE", "WRITE_SIZE"):
        f = pass_csv(name)
        rows = [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"] or "reduce" in r["Kernel_Name"]]
        with open(os.path.join(dst, f"pmc_{name}.csv"), "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    fetch_kb, write_kb = statistics.mean(fetch), statistics.mean(write)
    bytes_per_launch = int((2.0 * fetch_kb + write_kb) * 1024)
    stats = list(csv.DictReader(open(glob.glob(os.path.join(src, "prof", "**", "*kernel_stats.csv"), recursive=True)[0])))
    trace = [r for r in stats if "trace_kernel" in r["Name"]][0]
    out = {"workload": workload, "bvh": bvh, "kernel": "rt::trace_kernel",
           "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving), mean over the "
                         "trace_kernel dispatches of the pass",
           "dispatches": len(fetch),
           "hbm_bytes_per_launch": bytes_per_launch,
           "rocprof_avg_ns": float(trace["AverageNs"]), "rocprof_calls": int(trace["Calls"])}
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    if not os.environ.get("PMC_NO_TOP"):  # (a config other than the headline: keep profiles/traffic.json)
        json.dump(out, open(os.path.join(os.path.dirname(dst.rstrip("/")), "traffic.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:5])
