#!/bin/bash
# PMC passes of one 50-spp headline-geometry frame for a given engine (default split):
#   tools/diag_split.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-split}; shift
out=gpurun_out/diag_$tag
mkdir -p $out
args="--spp 50 --steps 1 --warmup 0 --no-cpu $@"
i=0
for set in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/p$i.log; exit $rc; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "split_kernel" in r["Kernel_Name"] or "trace_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
line = json.loads([l for l in open(out + "/p1.log") if l.startswith('{"metric"')][-1])
seg = line["roofline"]["segments_per_launch"]
for c in sorted(agg): print(f"   {c:28s} {agg[c]:.4g}   per segment {agg[c]/seg:.3f}")
w = agg["SQ_WAVE_CYCLES"]; v = agg["SQ_ACTIVE_INST_VALU"]
print("valu busy (4 waves/SIMD):", v / (w / 4), " lane util:", agg["SQ_THREAD_CYCLES_VALU"] / (64 * v), " Msamples/s:", line["value"])
PY
