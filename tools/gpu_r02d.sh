#!/bin/bash
# Round-2 session D: spill-fix headline bench, instruction-cost microbenchmark, wavefront diagnosis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-1500; return $rc; }
run bench_mk 300 python bench.py --steps 5 --warmup 1 --no-cpu || exit 1
run ubench 120 exp/ubench 768 || exit 1
run bench_wf 300 python bench.py --steps 2 --warmup 1 --no-cpu --engine wavefront --timing || exit 1
bash tools/diag_wf.sh wf --engine wavefront || exit 1
