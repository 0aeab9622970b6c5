#!/bin/bash
# Round-2 session Q: tile-major guided unit lengths with the 3x tail phase (main) vs the previous build
# (old) and the same kernel without guiding (g0): headline, per-rank frames N = 1/2/4/8, cfg1/earth.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=3 bash tools/ab2.sh "old;;" "g0;;" "main;;" "old;;" "g0;;" "main;;" || exit $?
for v in old main; do
  d=$PWD/exp/$v; [ $v = main ] && d=""
  SHIRLEY_LIB_DIR=$d timeout -k 10 300 python tools/shard_balance.py gpurun_out/sbq_$v.json --reps 2 > gpurun_out/sbq_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/sbq_$v.json')); print('$v', {w: (max(r['rank_kernel_ms']), r['sample_chunk'][0], r['predicted_efficiency']) for w, r in d['worlds'].items()})"
done
AB_STEPS=1 bash tools/ab2.sh "old;;--scene random --width 400 --aspect std16x9 --spp 50" "main;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "old;;--scene earth --width 800 --aspect square --spp 1000" "main;;--scene earth --width 800 --aspect square --spp 1000"
