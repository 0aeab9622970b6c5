# gen_spheres and cfg1 on the final build vs the build before box_t1f and the LDS material tables
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=10 AB_REPS=3 bash tools/gpu.sh r05z8a "ab:pre||$GS;main||$GS" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05z8b "ab:pre||$C1;main||$C1"
