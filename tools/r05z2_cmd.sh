# code object for gfx950:xnack- (the pool runs with XNACK off) vs the target-id-agnostic gfx950 build
CO="--scene cornell --width 600 --aspect square --spp 1000"
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05z2a "ab:main||;xn||;main||$CO;xn||$CO;main||$F;xn||$F;main||$GS;xn||$GS"
