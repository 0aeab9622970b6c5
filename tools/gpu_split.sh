#!/bin/bash
# RT_ENGINE_SPLIT bring-up: parity (bit-identical to the megakernel) first, then A/B benches of the
# traversal-wave count and the claim threshold on the headline frame.  Any failure stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-700; return $rc; }
run split_smoke 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "test_render_matches_oracle and random-48" || exit 1
run split_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k split || exit 1
run b_mk 200 python bench.py --steps 3 --warmup 1 --no-cpu --engine megakernel || exit 1
for nt in 8 6 4; do for rf in 8; do
  SHIRLEY_SPLIT_NT=$nt SHIRLEY_SPLIT_REFILL=$rf run b_split_${nt}_${rf} 200 python bench.py --steps 3 --warmup 1 --no-cpu --engine split || exit 1
done; done
for rf in 1 4 16 32; do
  SHIRLEY_SPLIT_NT=8 SHIRLEY_SPLIT_REFILL=$rf run b_split_8_${rf} 200 python bench.py --steps 3 --warmup 1 --no-cpu --engine split || exit 1
done
