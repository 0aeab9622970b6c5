#!/bin/bash
# Correctness gate for a kernel change (divcheck + parity/traversal subset), then an alternating A/B of
# the headline bench: exp/<base> vs the in-tree build.  Usage: tools/gpu_ab.sh [base] [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets  # variant libs live in exp/<name>/
base=${1:-base}; rounds=${2:-2}
timeout -k 10 120 shirley-raytracing-rs_amd/bin/divcheck 24 8 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_traversal.py tests/test_gpu_parity.py -k "traversal or render_matches or hit_queries or large_scene or edge or headline" > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq $rounds); do
  for v in $base main; do
    if [ $v = main ]; then dir=""; else dir="$PWD/exp/$v"; fi
    SHIRLEY_LIB_DIR=$dir timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs $BENCH_ARGS > gpurun_out/ab/$v.log 2>&1
    rc=$?
    echo "$r $v rc=$rc $(grep '^{"metric"' gpurun_out/ab/$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms")')"
    [ $rc -eq 0 ] || exit $rc
  done
done
