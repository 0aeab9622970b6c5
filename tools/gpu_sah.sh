#!/bin/bash
# A/B of the tree build: 32-bin vs exact-sweep SAH (SHIRLEY_SAH_SWEEP) x greedy vs DP 4-wide
# collapse (SHIRLEY_COLLAPSE_GREEDY), after the traversal / parity tests on the DP collapse.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sah
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_traversal.py tests/test_gpu_parity.py -k "traversal or sah or render_matches_oracle or large_scene" > gpurun_out/sah/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sah/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for cfg in "random:--spp 500" "final:--width 1920 --aspect std16x9 --spp 100" "spheres:--width 1920 --aspect std16x9 --spp 16"; do
  sc=${cfg%%:*}; a=${cfg#*:}
  for mode in binned_greedy binned_dp sweep_greedy sweep_dp; do
    unset SHIRLEY_SAH_SWEEP SHIRLEY_COLLAPSE_GREEDY
    case $mode in sweep*) export SHIRLEY_SAH_SWEEP=1;; esac
    case $mode in *greedy) export SHIRLEY_COLLAPSE_GREEDY=1;; esac
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --scene $sc $a > gpurun_out/sah/${sc}_$mode.log 2>&1
    rc=$?
    echo "$rep $sc $mode rc=$rc $(grep '^{"metric"' gpurun_out/sah/${sc}_$mode.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms nodes/seg", c["node_tests_per_segment"], "prims/seg", c["prim_tests_per_segment"])')"
    [ $rc -eq 0 ] || exit $rc
  done
done
done
