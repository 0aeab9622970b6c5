#!/bin/bash
# Round-2 session R: per-wave unit segments with work stealing (ws, RT_WAVE_SEGMENTS=1) vs the global
# queue (main, old = previous build): headline, per-rank frames, other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "old;;" "main;;" "ws;;" "old;;" "main;;" "ws;;" || exit $?
SHIRLEY_LIB_DIR=$PWD/exp/ws timeout -k 10 300 python tools/shard_balance.py gpurun_out/sbr_ws.json --reps 2 > gpurun_out/sbr_ws.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/sbr_ws.json')); print('ws', {w: (max(r['rank_kernel_ms']), r['sample_chunk'][0], r['predicted_efficiency']) for w, r in d['worlds'].items()})"
AB_STEPS=1 bash tools/ab2.sh "main;;--scene random --width 400 --aspect std16x9 --spp 50" "ws;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "main;;--scene earth --width 800 --aspect square --spp 1000" "ws;;--scene earth --width 800 --aspect square --spp 1000" \
  "main;;--scene cornell --width 600 --aspect square --spp 2000" "ws;;--scene cornell --width 600 --aspect square --spp 2000" \
  "main;;--scene final --width 1920 --aspect std16x9 --spp 400" "ws;;--scene final --width 1920 --aspect std16x9 --spp 400" \
  "main;;--scene spheres --width 1920 --aspect std16x9 --spp 400" "ws;;--scene spheres --width 1920 --aspect std16x9 --spp 400"
