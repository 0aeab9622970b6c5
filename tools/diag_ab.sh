#!/bin/bash
# PMC counters of the trace kernel for several library builds (exp/<v> or main)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
args="--spp 50 --steps 1 --warmup 0 --no-cpu"
for v in "$@"; do
  extra=""
  case $v in main) dir="";; main:*) dir=""; extra="--nodes ${v#main:}";; *) dir="$PWD/exp/$v";; esac
  out=gpurun_out/dab_${v//:/_}; mkdir -p $out; i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"; do
    i=$((i+1))
    SHIRLEY_LIB_DIR=$dir timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args $extra > $out/p$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v pass $i rc=$rc"; tail -3 $out/p$i.log; exit $rc; }
  done
  python3 - "$out" "$v" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], " ".join(f"{k}={agg[k]:.3g}" for k in sorted(agg)))
PY
done
