#!/bin/bash
# Round-2 session S: per-wave unit segments + shared tail queue (ws: 1/4 shared, ws8: 1/8, ws2: 1/2)
# vs the global queue (old = previous build): headline, per-rank frames, other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "old;;" "ws;;" "ws8;;" "ws2;;" "old;;" "ws;;" "ws8;;" "ws2;;" || exit $?
for v in ws ws8; do
SHIRLEY_LIB_DIR=$PWD/exp/$v timeout -k 10 300 python tools/shard_balance.py gpurun_out/sbs_$v.json --reps 2 > gpurun_out/sbs_$v.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/sbs_$v.json')); print('$v', {w: (max(r['rank_kernel_ms']), r['sample_chunk'][0], r['predicted_efficiency']) for w, r in d['worlds'].items()})"
done
AB_STEPS=1 bash tools/ab2.sh "old;;--scene random --width 400 --aspect std16x9 --spp 50" "ws;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "old;;--scene earth --width 800 --aspect square --spp 1000" "ws;;--scene earth --width 800 --aspect square --spp 1000" \
  "old;;--scene cornell --width 600 --aspect square --spp 2000" "ws;;--scene cornell --width 600 --aspect square --spp 2000" \
  "old;;--scene final --width 1920 --aspect std16x9 --spp 400" "ws;;--scene final --width 1920 --aspect std16x9 --spp 400" \
  "old;;--scene spheres --width 1920 --aspect std16x9 --spp 400" "ws;;--scene spheres --width 1920 --aspect std16x9 --spp 400"
