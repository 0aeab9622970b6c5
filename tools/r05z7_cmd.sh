# material / texture tables in LDS for the book-2 wide block too (nodes in LDS, primitives via L1/L2)
F="--scene final --width 1920 --aspect std16x9 --spp 200"
bash tools/gpu.sh r05z7t "tests:tests/test_gpu_parity.py tests/test_gpu_box2.py tests/test_scatter_kat.py tests/test_gpu_multi.py" &&
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05z7a "ab:main|SHIRLEY_NO_LDS_MATS=1|$F;main||$F"
