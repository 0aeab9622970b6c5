# pop loop: K stack entries read per trip (main: K = 2; pop1 = one per trip, the previous loop; pop4)
CO="--scene cornell --width 600 --aspect square --spp 1000"
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05p1 "ab:pop1||$GS;main||$GS;pop4||$GS;pop1||$F;main||$F;pop4||$F;bx2e||$F" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05p2 "ab:pop1||;main||;pop4||;pop1||$CO;main||$CO;pop4||$CO" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05p3 "ab:pop1||$C1;main||$C1;pop4||$C1"
