#!/bin/bash
# Round-2 session R: headline unit length 8 (auto) vs 5 / 6, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=5 bash tools/ab2.sh "main;;" "main;;--sample-chunk 5" "main;;--sample-chunk 6" "main;;" "main;;--sample-chunk 5" \
  "main;;--sample-chunk 6" "main;;" "main;;--sample-chunk 5" "main;;--sample-chunk 6"
