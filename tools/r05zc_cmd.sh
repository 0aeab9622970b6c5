# scene-in-LDS instance: material / texture tables read with ds_read (main) vs FLAT loads (pre)
CO="--scene cornell --width 600 --aspect square --spp 1000"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zca "ab:pre||;main||;pre||$CO;main||$CO" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05zcb "ab:pre||$C1;main||$C1" &&
bash tools/gpu.sh r05zcc "tests:tests/test_gpu_parity.py tests/test_scatter_kat.py tests/test_gpu_ties.py tests/test_gpu_box2.py"
