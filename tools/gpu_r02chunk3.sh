#!/bin/bash
# Round-2 session R: unit length on the large-spp configs (auto chunk: gen_spheres / final 1920x1080 @
# 2000 spp -> 61, Cornell 600x600 @ 10000 spp -> 54).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="--scene spheres --width 1920 --aspect std16x9 --spp 2000"
F="--scene final --width 1920 --aspect std16x9 --spp 2000"
C="--scene cornell --width 600 --aspect square --spp 10000"
AB_STEPS=1 bash tools/ab2.sh "main;;$S" "main;;$S --sample-chunk 4" "main;;$S --sample-chunk 8" "main;;$S --sample-chunk 16" \
  "main;;$S --sample-chunk 32" "main;;$F" "main;;$F --sample-chunk 8" "main;;$F --sample-chunk 16" \
  "main;;$C" "main;;$C --sample-chunk 8" "main;;$C --sample-chunk 16" "main;;$C --sample-chunk 32"
