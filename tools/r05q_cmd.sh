# book-2 256-thread instances (scenes whose tree does not fit the wide block's LDS): 3 waves per SIMD
# (168 VGPRs) vs 4 (128 VGPRs, ~90 spilled); final_scene forced onto them with SHIRLEY_NO_WIDE; plus the
# book-2 parity tests on the default build (two-pass RectBox test in the book-2 instances)
F="--scene final --width 1920 --aspect std16x9 --spp 200"
bash tools/gpu.sh r05q0 "tests:tests/test_gpu_parity.py tests/test_scatter_kat.py tests/test_gpu_ties.py" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05q1 "ab:main|SHIRLEY_NO_WIDE=1|$F;nw3|SHIRLEY_NO_WIDE=1|$F" &&
bash tools/gpu.sh r05q2 "sh:SHIRLEY_NO_WIDE=1 SHIRLEY_LIB_DIR=$PWD/exp/nw3 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -k final -x -q -p no:cacheprovider"
