# material and texture tables in the scene-in-LDS block (SHIRLEY_LDS_MATS=1) vs global memory
CO="--scene cornell --width 600 --aspect square --spp 1000"
C1="--width 400 --aspect std16x9 --spp 50"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05z5a "ab:main||;main|SHIRLEY_LDS_MATS=1|;main||$CO;main|SHIRLEY_LDS_MATS=1|$CO" &&
AB_STEPS=20 AB_REPS=2 bash tools/gpu.sh r05z5b "ab:main||$C1;main|SHIRLEY_LDS_MATS=1|$C1" &&
bash tools/gpu.sh r05z5c "sh:SHIRLEY_LDS_MATS=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k 'render_matches_oracle or golden or settings_band'"
