cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export SHIRLEY_ASSETS=$PWD/shirley-raytracing-rs_amd/assets
V=${V:-boxskip}
SHIRLEY_LIB_DIR=$PWD/exp/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$V.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/parity_$V.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=5 bash tools/ab2.sh "prev;;" "$V;;" "prev;;" "$V;;" "prev;;--scene cornell --width 600 --aspect square --spp 500" "$V;;--scene cornell --width 600 --aspect square --spp 500"
