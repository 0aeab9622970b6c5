#!/bin/bash
# GPU parity tests, headline bench (regression check) and a book-2 final_scene bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
true

timeout -k 10 300 python bench.py --scene final --width 800 --aspect square --spp 100 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_final.log 2>&1 || exit 1
tail -1 gpurun_out/bench_final.log | cut -c1-600
