# optimal 4-wide collapse (SHIRLEY_COLLAPSE_DP) on the scene-in-LDS scenes: headline, Cornell, cfg1
CO="--scene cornell --width 600 --aspect square --spp 1000"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=4 bash tools/gpu.sh r05zga "ab:main||;main|SHIRLEY_COLLAPSE_DP=1|;main||$CO;main|SHIRLEY_COLLAPSE_DP=1|$CO" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05zgb "ab:main||$C1;main|SHIRLEY_COLLAPSE_DP=1|$C1"
