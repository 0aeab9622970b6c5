#!/bin/bash
# A/B of the 256-thread trace instances' occupancy: book-2 final_scene (EXT kernels) and gen_spheres
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/narrow
export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets  # variant libs live in exp/<name>/
for r in 1 2; do
for cfg in "final:--width 1920 --aspect std16x9 --spp 200" "spheres:--width 1920 --aspect std16x9 --spp 200"; do
  sc=${cfg%%:*}; a=${cfg#*:}
  for v in main e3 e2 n3; do
    if [ $v = main ]; then dir=""; else dir="$PWD/exp/$v"; fi
    SHIRLEY_LIB_DIR=$dir timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-configs --scene $sc $a > gpurun_out/narrow/${sc}_$v.log 2>&1
    rc=$?
    echo "$r $sc $v rc=$rc $(grep '^{"metric"' gpurun_out/narrow/${sc}_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms")')"
    [ $rc -eq 0 ] || exit $rc
  done
done
done
