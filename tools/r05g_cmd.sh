C1="--width 400 --aspect std16x9 --spp 50"
bash tools/gpu.sh r05g "tests:tests/test_gpu_parity.py tests/test_gpu_ranges.py tests/test_gpu_multi.py tests/test_scatter_kat.py tests/test_gpu_ties.py" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05g1 "ab:pre|SHIRLEY_QUEUE_TAIL=0|$C1;main||$C1" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05g2 "ab:pre||;main||" "sh:python tools/shard_balance.py gpurun_out/r05g2/shard_balance.json --reps 2" &&
bash tools/r05e_cmd.sh
