#!/bin/bash
# VALU lane utilisation and instruction mix of the trace kernel (reduced-spp headline frame)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/diag2_${1:-a}; shift
mkdir -p $out
args="--spp 50 --steps 1 --warmup 0 --no-cpu $@"
i=0
for set in "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/p$i.log; exit $rc; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg): print(f"{k:28s} {agg[k]:.4g}")
if agg.get("SQ_ACTIVE_INST_VALU"):
    print("VALUUtilization %.1f %%" % (100 * agg["SQ_THREAD_CYCLES_VALU"] / (agg["SQ_ACTIVE_INST_VALU"] * 64)))
PY
