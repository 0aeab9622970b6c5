# sphere leaves read through L1/L2: the next leaf's first word loaded during the current test (spf)
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=10 AB_REPS=2 bash tools/gpu.sh r05s1 "ab:main||$GS;spf||$GS" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05s2 "ab:main||$F;spf||$F"
