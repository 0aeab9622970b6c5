#!/bin/bash
# Round-2 session F (HEAD re-validation after the container re-creation): whole -m gpu suite,
# smoke, headline bench with CPU baseline, rocprof kernel trace + HBM PMC, VALU PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SHIRLEY_PARITY_LOG=$PWD/gpurun_out/parity_fractions.jsonl
rm -f "$SHIRLEY_PARITY_LOG"
run() { local name=$1 secs=$2; shift 2; echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
run gpu_tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench_full 400 python bench.py --steps 5 --warmup 1 || exit 1
bash tools/profile.sh r02 --steps 2 --warmup 1 --no-cpu --no-configs || exit 1
bash tools/profile_valu.sh r02 || exit 1
