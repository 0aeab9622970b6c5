#!/bin/bash
# Round-2 session I: -m gpu suite (incl. the bench's config-5 sharded leg on a one-rank job), the VALU
# PMC passes of the current build (profiles/r02/valu.json), and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/i_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/i_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_valu.sh r02 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/i_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/i_bench.log | cut -c1-300
