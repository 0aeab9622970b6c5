F="--scene final --width 1920 --aspect std16x9 --spp 200"
bash tools/gpu.sh r05j tests &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05j1 "ab:pre||$F;main||$F"
