#!/bin/bash
# wavefront bring-up: new engine tests first, then both engines on the headline config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "wavefront or render_matches" > gpurun_out/wf_tests.log 2>&1
rc=$?; echo "wf tests rc=$rc"; tail -15 gpurun_out/wf_tests.log
[ $rc -eq 0 ] || exit $rc
for e in megakernel wavefront; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --engine $e --timing "$@" > gpurun_out/bench_$e.log 2>&1; rc=$?
  echo "$e rc=$rc"; tail -1 gpurun_out/bench_$e.log | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
done
