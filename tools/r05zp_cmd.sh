# weighted sweep SAH by default (RectBox 4): main vs the previous build (pre) on Cornell, headline, final,
# gen_spheres, cfg1; then the whole GPU suite
CO="--scene cornell --width 600 --aspect square --spp 1000"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
S="--scene spheres --width 1920 --aspect std16x9 --spp 200"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zpa "ab:pre||$CO;main||$CO;pre||;main||;pre||$F;main||$F;pre||$S;main||$S" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05zpb "ab:pre||$C1;main||$C1" &&
bash tools/gpu.sh r05zpc tests
