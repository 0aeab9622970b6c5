#!/bin/bash
# Round-2 GPU session: new traversal / settings / config-5 tests, the whole -m gpu suite, headline
# bench with the CPU baseline, VALU PMC.  Each GPU step has its own time limit; a crash / timeout
# stops the session (test failures do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SHIRLEY_PARITY_LOG=$PWD/gpurun_out/parity_fractions.jsonl
rm -f "$SHIRLEY_PARITY_LOG"
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  return $rc
}
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
run new_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_traversal.py tests/test_gpu_parity.py -k "traversal or headline or max_depth or world8 or side11"
ok $? || exit 1
run gpu_tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
ok $? || exit 1
run bench_full 400 python bench.py --steps 3 --warmup 1 || exit 1
bash tools/profile_valu.sh r02 || exit 1
