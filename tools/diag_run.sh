cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHIRLEY_LIB_DIR=$PWD/exp/phase timeout -k 10 300 python bench.py --spp 100 --steps 1 --warmup 1 --no-cpu > gpurun_out/phase.log 2>&1; echo rc=$?
grep phase gpurun_out/phase.log
bash tools/diag.sh cur 2>&1 | tail -30
