cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scene final --width 1920 --aspect std16x9 --spp 2000 --steps 1 --warmup 1 --no-cpu > gpurun_out/bench_cfg5.log 2>&1; echo "cfg5 rc=$?"; tail -1 gpurun_out/bench_cfg5.log | cut -c1-700
