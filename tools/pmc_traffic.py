"""Summarise a tools/profile.sh run: kernel-trace stats + per-dispatch HBM traffic of the trace
kernel from the FETCH_SIZE / WRITE_SIZE passes, corrected as MI355X_MICROARCH.md §HBM prescribes
(counters in KiB; gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads -> x2).
Writes profiles/<tag>/ (copied CSV summaries) and profiles/traffic.json (read by bench.py).

usage: python tools/pmc_traffic.py <gpurun_out/prof_TAG> <profiles/TAG> <workload> <bvh>
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
    for f in glob.glob(os.path.join(src, "trace", "*kernel_stats.csv")) + \
            glob.glob(os.path.join(src, "trace", "*domain_stats.csv")):
        shutil.copy(f, os.path.join(dst, os.path.basename(f).replace("run_", "")))
    fetch = per_dispatch(glob.glob(os.path.join(src, "pmc_FETCH_SIZE", "*counter_collection.csv"))[0], "trace_kernel")
    write = per_dispatch(glob.glob(os.path.join(src, "pmc_WRITE_SIZE", "*counter_collection.csv"))[0], "trace_kernel")
    for name in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(src, f"pmc_{name}", "*counter_collection.csv"))[0]
        rows = [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"] or "reduce" in r["Kernel_Name"]]
        with open(os.path.join(dst, f"pmc_{name}.csv"), "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    fetch_kb, write_kb = statistics.median(fetch), statistics.median(write)
    bytes_per_launch = int((2.0 * fetch_kb + write_kb) * 1024)
    stats = list(csv.DictReader(open(glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0])))
    trace = [r for r in stats if "trace_kernel" in r["Name"]][0]
    out = {"workload": workload, "bvh": bvh, "kernel": "rt::trace_kernel",
           "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
           "hbm_bytes_per_launch": bytes_per_launch,
           "rocprof_avg_ns": float(trace["AverageNs"]), "rocprof_calls": int(trace["Calls"])}
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(os.path.dirname(dst.rstrip("/")), "traffic.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:5])
