#!/bin/bash
# VALU PMC passes of one headline-geometry frame (bench --steps 1 --warmup 0: one trace_kernel
# dispatch per pass), then tools/pmc_valu.py -> profiles/<tag>/valu.json + profiles/valu.json.
# Usage: tools/profile_valu.sh <tag> [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r02}; shift
out=gpurun_out/valu_$tag
mkdir -p $out
args="--spp 50 --steps 1 --warmup 0 --no-cpu --no-configs --bvh sah $@"
i=0
for set in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/p$i.log; exit $rc; }
done
python3 tools/pmc_valu.py profiles/$tag 4 $out/p1
