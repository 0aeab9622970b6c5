#!/bin/bash
# Round-2 session G: the -m gpu suite on the in-tree build, then A/B of experiment variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/g_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/g_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=3 bash tools/ab2.sh "$@"
