#!/bin/bash
# Round-2 final check on HEAD's build: -m gpu suite, smoke(), the default bench line, rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/z_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/z_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/z_bench.log 2>&1 || exit $?
tail -1 gpurun_out/z_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-configs \
  > gpurun_out/z_prof.log 2>&1 || exit $?
tail -1 gpurun_out/z_prof.log | cut -c1-200
find gpurun_out/z_prof -name "*kernel_stats.csv"
