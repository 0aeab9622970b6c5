#!/bin/bash
# Round-2 session R: sample_chunk scan on the block-segment build (headline frame; auto = 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "main;;" "main;;--sample-chunk 10" "main;;--sample-chunk 16" "main;;--sample-chunk 25" \
  "main;;--sample-chunk 50" "main;;" "main;;--sample-chunk 16" "main;;--sample-chunk 32" || exit $?
AB_STEPS=1 bash tools/ab2.sh "main;;--scene spheres --width 1920 --aspect std16x9 --spp 2000" \
  "main;;--scene spheres --width 1920 --aspect std16x9 --spp 2000 --sample-chunk 64" \
  "main;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000 --sample-chunk 32" \
  "main;;--scene cornell --width 600 --aspect square --spp 2000" "main;;--scene cornell --width 600 --aspect square --spp 2000 --sample-chunk 16"
