#!/bin/bash
# Round-2 session L: guided unit lengths (long chunks, then one-sample units at the end of the pool) —
# -m gpu suite on the in-tree build, A/B against the previous build (exp/old) on the headline, the
# per-rank frames of N = 1/2/4/8 (tools/shard_balance.py) and the other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/l_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/l_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "old;;" "main;;" "old;;" "main;;" || exit $?
SHIRLEY_LIB_DIR=$PWD/exp/old timeout -k 10 300 python tools/shard_balance.py gpurun_out/sb_old.json --reps 2 > gpurun_out/sb_old.log 2>&1 || exit $?
timeout -k 10 300 python tools/shard_balance.py gpurun_out/sb_main.json --reps 2 > gpurun_out/sb_main.log 2>&1 || exit $?
tail -n 6 gpurun_out/sb_old.log gpurun_out/sb_main.log
AB_STEPS=2 bash tools/ab2.sh "old;;--scene random --width 400 --aspect std16x9 --spp 50" "main;;--scene random --width 400 --aspect std16x9 --spp 50" \
  "old;;--scene final --width 1920 --aspect std16x9 --spp 200" "main;;--scene final --width 1920 --aspect std16x9 --spp 200" \
  "old;;--scene cornell --width 600 --aspect square --spp 1000" "main;;--scene cornell --width 600 --aspect square --spp 1000" \
  "old;;--scene spheres --width 1920 --aspect std16x9 --spp 200" "main;;--scene spheres --width 1920 --aspect std16x9 --spp 200"
