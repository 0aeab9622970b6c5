#!/bin/bash
# Per-kernel diagnosis (kernel trace + PMC passes) of a reduced-spp headline frame.
#   tools/diag_wf.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/diag_${1:-a}; shift
mkdir -p $out
args="--spp 64 --steps 1 --warmup 0 --no-cpu $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 bench.py $args > $out/kt.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/kt.log; exit $rc; }
tail -1 $out/kt.log | cut -c1-300
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_ATOMIC_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/p$i.log; [ $rc -eq 1 ] || exit $rc; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections, re
out = sys.argv[1]
for f in glob.glob(out + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} total_ms {float(r["TotalDurationNs"])/1e6:9.2f} avg_us {float(r["AverageNs"])/1e3:9.2f}')
agg = collections.defaultdict(lambda: collections.defaultdict(float))
def short(n):
    m = re.search(r"(wf_\w+|trace_kernel|reduce_kernel|hit_kernel|unpack_kernel)", n)
    return m.group(1) if m else "other"
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    if k == "other": continue
    print("==", k)
    for c in sorted(agg[k]): print(f"   {c:28s} {agg[k][c]:.4g}")
PY
