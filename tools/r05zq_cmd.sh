# weighted sweep SAH for book-2 objects (SHIRLEY_SAH_EXTW: instances, media, moving spheres weigh c) on final_scene
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05zqa "ab:main||$F;main|SHIRLEY_SAH_EXTW=2|$F;main|SHIRLEY_SAH_EXTW=4|$F;main|SHIRLEY_SAH_BOXW=1|$F"
