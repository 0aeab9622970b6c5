cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets
SHIRLEY_LIB_DIR=$PWD/exp/slds timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "render_matches_oracle and random" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_slds.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/parity_slds.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=5 bash tools/ab2.sh "prev;;" "slds;;" "prev;;" "slds;;" "prev;;" "slds;;"
