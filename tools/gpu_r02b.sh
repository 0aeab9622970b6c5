#!/bin/bash
# Round-2 GPU session B: multi-GPU ABI tests, full -m gpu suite, bench, shard balance.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  return $rc
}
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
run multi_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py
ok $? || exit 1
run gpu_tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
ok $? || exit 1
run bench_full 400 python bench.py --steps 5 --warmup 1 --no-cpu || exit 1
run shard_balance 300 python tools/shard_balance.py gpurun_out/shard_balance.json || exit 1
