#!/bin/bash
# book-2 final_scene: 1024-thread EXT instance (4 waves/SIMD, ~80 spilled VGPRs) vs 768 threads
# (3 waves/SIMD, no spills; SHIRLEY_WIDE3).  Parity of the 768 path first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wide3
SHIRLEY_WIDE3=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_traversal.py tests/test_book2_ext.py -k "final" > gpurun_out/wide3/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/wide3/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  if [ $v = 1 ]; then export SHIRLEY_WIDE3=1; else unset SHIRLEY_WIDE3; fi
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-configs --scene final --width 1920 --aspect std16x9 --spp 200 > gpurun_out/wide3/b$v.log 2>&1
  rc=$?
  echo "$r wide3=$v rc=$rc $(grep '^{"metric"' gpurun_out/wide3/b$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms")')"
  [ $rc -eq 0 ] || exit $rc
done; done
