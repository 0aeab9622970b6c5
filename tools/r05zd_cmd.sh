# no FLAT loads left in the scene-in-LDS instance: the sphere leaf's primitive re-read laundered as an LDS
# pointer, image texels typed global (main) vs the previous build (pre)
CO="--scene cornell --width 600 --aspect square --spp 1000"
E="--scene earth --width 800 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zda "ab:pre||;main||;pre||$CO;main||$CO;pre||$E;main||$E" &&
bash tools/gpu.sh r05zdc "tests:tests/test_gpu_parity.py tests/test_scatter_kat.py tests/test_divisions.py"
