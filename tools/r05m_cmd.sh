# book-2 instances: scene record from the KBlock per iteration (SGPR spills 50 -> 25) vs held in SGPRs
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05m1 "ab:main||$F;exks||$F" &&
bash tools/gpu.sh r05m2 "testsv:exks:tests/test_gpu_parity.py -k final"
