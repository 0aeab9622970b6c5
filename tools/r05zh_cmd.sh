# the optimal 4-wide collapse for scene-in-LDS reference scenes (greedy elsewhere): main vs the previous
# build (pre) on the headline, Cornell, gen_spheres, cfg1, then the whole GPU suite
CO="--scene cornell --width 600 --aspect square --spp 1000"
S="--scene spheres --width 1920 --aspect std16x9 --spp 200"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zha "ab:pre||;main||;pre||$CO;main||$CO;pre||$S;main||$S" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05zhb "ab:pre||$C1;main||$C1" &&
bash tools/gpu.sh r05zhc tests
