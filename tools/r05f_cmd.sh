C1="--width 400 --aspect std16x9 --spp 50"
SP="--scene spheres --width 1920 --aspect std16x9 --spp 200"
bash tools/gpu.sh r05f "tests:tests/test_gpu_parity.py tests/test_gpu_ranges.py tests/test_gpu_multi.py" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05f1 "ab:pre|SHIRLEY_QUEUE_TAIL=0|$C1;main||$C1;main|SHIRLEY_QUEUE_TAIL=0|$C1;main|SHIRLEY_WINDOW=64|$C1;main|SHIRLEY_QUEUE_TAIL=2097152|$C1;main|SHIRLEY_QUEUE_TAIL=524288|$C1" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05f2 "ab:pre||;main||;surelds||;pre||$SP;main||$SP;surelds||$SP" "sh:python tools/shard_balance.py gpurun_out/r05f2/sb_main.json --worlds 8 --partitions tiles,samples --reps 2"
