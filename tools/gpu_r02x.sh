#!/bin/bash
# Round-2 re-entry check on a rebuilt tree: -m gpu suite, smoke(), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/x_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/x_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/x_bench.log 2>&1 || exit $?
tail -1 gpurun_out/x_bench.log
