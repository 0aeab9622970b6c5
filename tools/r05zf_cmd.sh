# optimal 4-wide collapse (SHIRLEY_COLLAPSE_DP) re-measured on this round's kernel: gen_spheres, final, headline
S="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05zfa "ab:main||$S;main|SHIRLEY_COLLAPSE_DP=1|$S;main||$F;main|SHIRLEY_COLLAPSE_DP=1|$F;main||;main|SHIRLEY_COLLAPSE_DP=1|"
