#!/bin/bash
# Round-2 session T: per-block unit segments with parallel-scan stealing (bs, RT_BLOCK_SEGMENTS=1) vs
# the global queue (old): parity subset on bs, headline, per-rank frames, other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets SHIRLEY_LIB_DIR=$PWD/exp/bs timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "headline_settings or config_settings or tiles_gather or scanlines or max_depth or edge_cases or render_matches_oracle" \
  > gpurun_out/t_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/t_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "old;;" "bs;;" "old;;" "bs;;" || exit $?
SHIRLEY_LIB_DIR=$PWD/exp/bs timeout -k 10 300 python tools/shard_balance.py gpurun_out/sbt_bs.json --reps 2 > gpurun_out/sbt_bs.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/sbt_bs.json')); print('bs', {w: (max(r['rank_kernel_ms']), r['sample_chunk'][0], r['predicted_efficiency']) for w, r in d['worlds'].items()})"
AB_STEPS=1 bash tools/ab2.sh "old;;--scene random --width 400 --aspect std16x9 --spp 50" "bs;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "old;;--scene earth --width 800 --aspect square --spp 1000" "bs;;--scene earth --width 800 --aspect square --spp 1000" \
  "old;;--scene cornell --width 600 --aspect square --spp 2000" "bs;;--scene cornell --width 600 --aspect square --spp 2000" \
  "old;;--scene final --width 1920 --aspect std16x9 --spp 400" "bs;;--scene final --width 1920 --aspect std16x9 --spp 400" \
  "old;;--scene spheres --width 1920 --aspect std16x9 --spp 400" "bs;;--scene spheres --width 1920 --aspect std16x9 --spp 400"
