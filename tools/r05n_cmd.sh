# book-2 hit record without the scratch-resident u, v (ext_record fills one record per branch)
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05n1 "ab:pre||$F;main||$F" &&
bash tools/gpu.sh r05n2 "tests:tests/test_gpu_parity.py tests/test_scatter_kat.py"
