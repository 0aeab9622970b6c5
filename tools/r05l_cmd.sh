# box_t2 straight-line (pass 2 re-reads the box) against the six-face test
C1="--width 400 --aspect std16x9 --spp 50"
CO="--scene cornell --width 600 --aspect square --spp 1000"
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05l1 "ab:six||;main||;six||$CO;main||$CO;six||$F;main||$F" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05l2 "ab:six||$C1;main||$C1;six||$GS;main||$GS"
