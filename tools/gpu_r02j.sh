#!/bin/bash
# Round-2 session J: dielectric chaining (traverse4_chain) — -m gpu suite on the in-tree build (chain 2),
# then A/B of chain depths 0 (off) / 1 / 2 (main) / 3 / 4 on the headline and the other scenes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/j_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/j_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "c0;;" "main;;" "c1;;" "c3;;" "c4;;" "c0;;" "main;;" || exit $?
AB_STEPS=1 bash tools/ab2.sh "c0;;--scene cornell --width 600 --aspect square --spp 1000" \
  "main;;--scene cornell --width 600 --aspect square --spp 1000" \
  "c0;;--scene final --width 1920 --aspect std16x9 --spp 200" "main;;--scene final --width 1920 --aspect std16x9 --spp 200" \
  "c0;;--scene spheres --width 1920 --aspect std16x9 --spp 200" "main;;--scene spheres --width 1920 --aspect std16x9 --spp 200" \
  "c0;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000"
