# box_t1f kept out of the L1/L2 reference instances (gen_spheres) vs the previous build
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=10 AB_REPS=3 bash tools/gpu.sh r05z9a "ab:pre||$GS;main||$GS" && AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05z9b "ab:main||"
