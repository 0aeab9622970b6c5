# weighted sweep SAH: a RectBox leaf weighs c (SHIRLEY_SAH_BOXW) in the split cost — Cornell and headline
CO="--scene cornell --width 600 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05zoa "ab:main||$CO;main|SHIRLEY_SAH_BOXW=2|$CO;main|SHIRLEY_SAH_BOXW=4|$CO;main|SHIRLEY_SAH_BOXW=8|$CO;main||;main|SHIRLEY_SAH_BOXW=2|;main|SHIRLEY_SAH_BOXW=4|;main|SHIRLEY_SAH_BOXW=8|"
