#!/bin/bash
# Round-2 session R: one Philox call site in draws_coop (donor lanes evaluate block B for lanes that
# need two blocks) — parity suite on exp/donor, then A/B against the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets SHIRLEY_LIB_DIR=$PWD/exp/donor timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/y_tests.log 2>&1
rc=$?; echo "donor parity rc=$rc"; tail -n 3 gpurun_out/y_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "main;;" "donor;;" "main;;" "donor;;" "main;;" "donor;;" || exit $?
AB_STEPS=1 bash tools/ab2.sh "main;;--scene cornell --width 600 --aspect square --spp 1000" \
  "donor;;--scene cornell --width 600 --aspect square --spp 1000" \
  "main;;--scene final --width 1920 --aspect std16x9 --spp 200" "donor;;--scene final --width 1920 --aspect std16x9 --spp 200" \
  "main;;--scene spheres --width 1920 --aspect std16x9 --spp 200" "donor;;--scene spheres --width 1920 --aspect std16x9 --spp 200" \
  "main;;--scene earth --width 800 --aspect square --spp 1000" "donor;;--scene earth --width 800 --aspect square --spp 1000"
