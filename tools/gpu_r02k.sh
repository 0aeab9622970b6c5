#!/bin/bash
# Round-2 session K: dielectric chaining gated on short traversals (RT_CHAIN_STEPS) — A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "c0;;" "main;;" "s1c3;;" "s1c4;;" "s2c2;;" "c0;;" "main;;" || exit $?
AB_STEPS=1 bash tools/ab2.sh "c0;;--scene cornell --width 600 --aspect square --spp 1000" \
  "main;;--scene cornell --width 600 --aspect square --spp 1000" \
  "c0;;--scene spheres --width 1920 --aspect std16x9 --spp 200" "main;;--scene spheres --width 1920 --aspect std16x9 --spp 200" \
  "c0;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000"
