# two-pass RectBox test (box_t2) against the six-face test: parity, then A/B on every headline-adjacent frame
C1="--width 400 --aspect std16x9 --spp 50"
CO="--scene cornell --width 600 --aspect square --spp 1000"
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
bash tools/gpu.sh r05k "tests:tests/test_gpu_parity.py tests/test_scatter_kat.py tests/test_gpu_ties.py tests/test_gpu_ranges.py" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05k1 "ab:six||;main||;six||$CO;main||$CO;six||$F;main||$F" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05k2 "ab:six||$C1;main||$C1;six||$GS;main||$GS"
