# tail units: the last samples of each pixel in one-sample chunks served last by every segment
CO="--scene cornell --width 600 --aspect square --spp 1000"
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05y1 "ab:main|SHIRLEY_TAIL=0|;main||;main|SHIRLEY_TAIL=32|;main|SHIRLEY_TAIL=8|" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05y2 "ab:main|SHIRLEY_TAIL=0|$CO;main||$CO;main|SHIRLEY_TAIL=0|$F;main||$F;main|SHIRLEY_TAIL=0|$GS;main||$GS" &&
bash tools/gpu.sh r05y3 "tests:tests/test_gpu_ranges.py tests/test_gpu_multi.py tests/test_gpu_parity.py"
