#!/bin/bash
# Round-2 session O: the new config-band parity tests in the full -m gpu suite; timeline of an N = 8
# rank frame (per-wave start / pool-dry / exit stamps) at auto chunk (1), chunk 2 and chunk 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/o_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/o_tests.log; [ $rc -eq 0 ] || exit $rc
for ch in 0 2 8; do
  SHIRLEY_LIB_DIR=$PWD/exp/tl timeout -k 10 300 python tools/shard_balance.py gpurun_out/tl_$ch.json --worlds 1,8 --reps 1 --chunk $ch \
    > gpurun_out/tl_$ch.log 2>&1 || exit $?
  grep -h "phase-timeline\|world" gpurun_out/tl_$ch.log | head -4
done
