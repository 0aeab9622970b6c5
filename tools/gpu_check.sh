#!/bin/bash
# full GPU test suite on the in-tree build, then an interleaved A/B against exp/<variant>s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB_STEPS=${AB_STEPS:-5} bash tools/ab2.sh "$@"
