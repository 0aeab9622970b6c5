# reference-scene instance: near-plane pass with a six-face fallback (b1f) vs the six-face sequence
CO="--scene cornell --width 600 --aspect square --spp 1000"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05z3a "ab:main||;b1f||;main||$CO;b1f||$CO" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05z3b "ab:main||$C1;b1f||$C1" &&
bash tools/gpu.sh r05z3c "testsv:b1f:tests/test_gpu_parity.py tests/test_gpu_box2.py tests/test_gpu_ties.py"
