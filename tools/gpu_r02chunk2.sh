#!/bin/bash
# Round-2 session R: sample_chunk below the auto choice (8) on the headline frame, i.e. past the 2 GiB
# partial-buffer cap (chunk 4 = 2.9 GB), and on the other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "main;;" "main;;--sample-chunk 4" "main;;--sample-chunk 5" "main;;--sample-chunk 6" \
  "main;;--sample-chunk 7" "main;;" "main;;--sample-chunk 4" "main;;--sample-chunk 2" || exit $?
AB_STEPS=1 bash tools/ab2.sh "main;;--scene spheres --width 1920 --aspect std16x9 --spp 2000" \
  "main;;--scene spheres --width 1920 --aspect std16x9 --spp 2000 --sample-chunk 8" \
  "main;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000 --sample-chunk 4" \
  "main;;--scene cornell --width 600 --aspect square --spp 2000" "main;;--scene cornell --width 600 --aspect square --spp 2000 --sample-chunk 4" \
  "main;;--scene final --width 1920 --aspect std16x9 --spp 400" "main;;--scene final --width 1920 --aspect std16x9 --spp 400 --sample-chunk 4"
grep -h '"sample_chunk"\|n_chunks' gpurun_out/ab2_*.log | head -3
