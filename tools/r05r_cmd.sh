# reference-scene 256-thread instances (gen_spheres: tree via L1/L2) at 3 waves per SIMD vs 4
bash tools/gpu.sh r05r0 "tests:tests/test_gpu_parity.py -k narrow_block" &&
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=10 AB_REPS=2 bash tools/gpu.sh r05r1 "ab:main||$GS;nw3r||$GS" &&
CO="--scene cornell --width 600 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05r2 "ab:main||;w3r|SHIRLEY_WIDE3_REF=1|;main||$CO;w3r|SHIRLEY_WIDE3_REF=1|$CO"
