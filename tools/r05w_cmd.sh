# reduce kernel with 8 chunks' loads in flight (main) vs one chunk per trip (prered): N=1 and the 8-rank shares
bash tools/gpu.sh r05w1 "sh:python tools/shard_balance.py gpurun_out/r05w1/main.json --reps 2 --worlds 1,8 --partitions tiles,samples" &&
bash tools/gpu.sh r05w2 "sh:SHIRLEY_LIB_DIR=$PWD/exp/prered python tools/shard_balance.py gpurun_out/r05w2/pre.json --reps 2 --worlds 1,8 --partitions tiles,samples" &&
bash tools/gpu.sh r05w3 "tests:tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_ranges.py"
