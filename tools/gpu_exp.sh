#!/bin/bash
# experiment session: instruction costs, A/B of library variants, parity of a candidate variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets
if [ -x exp/ubench ]; then timeout -k 10 120 exp/ubench 768 > gpurun_out/ubench.log 2>&1; echo "ubench rc=$?"; cat gpurun_out/ubench.log; fi
if [ -n "$PARITY_VARIANT" ]; then
  SHIRLEY_LIB_DIR=$PWD/exp/$PARITY_VARIANT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$PARITY_VARIANT.log 2>&1
  rc=$?; echo "parity($PARITY_VARIANT) rc=$rc"; tail -3 gpurun_out/parity_$PARITY_VARIANT.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
AB_STEPS=${AB_STEPS:-3} bash tools/ab2.sh "$@"
