#!/bin/bash
# Round-2 session U: per-block unit segments for units of >= 4 samples (in-tree build) — -m gpu suite,
# A/B against the previous build (old), per-rank frames, other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/u_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/u_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "old;;" "main;;" "old;;" "main;;" || exit $?
timeout -k 10 300 python tools/shard_balance.py gpurun_out/sbu_main.json --reps 2 > gpurun_out/sbu_main.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/sbu_main.json')); print('main', {w: (max(r['rank_kernel_ms']), r['sample_chunk'][0], r['predicted_efficiency']) for w, r in d['worlds'].items()})"
AB_STEPS=1 bash tools/ab2.sh "old;;--scene random --width 400 --aspect std16x9 --spp 50" "main;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "old;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000" \
  "old;;--scene cornell --width 600 --aspect square --spp 2000" "main;;--scene cornell --width 600 --aspect square --spp 2000" \
  "old;;--scene final --width 1920 --aspect std16x9 --spp 400" "main;;--scene final --width 1920 --aspect std16x9 --spp 400" \
  "old;;--scene spheres --width 1920 --aspect std16x9 --spp 400" "main;;--scene spheres --width 1920 --aspect std16x9 --spp 400"
