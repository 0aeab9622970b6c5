#!/bin/bash
# Round-2 session R: unit length on the small cfg1 frame (random 400x225 @ 50 spp; auto chunk 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="--scene random --width 400 --aspect std16x9 --spp 50"
AB_STEPS=20 bash tools/ab2.sh "main;;$A" "main;;$A --sample-chunk 2" "main;;$A --sample-chunk 3" "main;;$A --sample-chunk 4" \
  "main;;$A --sample-chunk 5" "main;;$A" "main;;$A --sample-chunk 2" "main;;$A --sample-chunk 4"
