# side_draw's round keys pinned to SGPRs like philox10 (book-2 instances: 31 -> 15 spilled SGPRs):
# main vs the previous build (pre) on the book-2 scenes
F="--scene final --width 1920 --aspect std16x9 --spp 200"
D="--scene demo --width 800 --aspect std16x9 --spp 500"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zea "ab:pre||$F;main||$F;pre||$D;main||$D" &&
bash tools/gpu.sh r05zec "tests:tests/test_gpu_parity.py tests/test_gpu_box2.py tests/test_scatter_kat.py"
