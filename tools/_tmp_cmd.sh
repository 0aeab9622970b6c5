cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets
SHIRLEY_LIB_DIR=$PWD/exp/ccam timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_ccam.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/parity_slds.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=5 bash tools/ab2.sh "prev;;" "ccam;;" "prev;;" "ccam;;" "prev;;" "ccam;;"
