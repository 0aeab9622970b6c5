# RectBox face test in the reference-scene instance re-ranked on the new Cornell tree: box_t1f (main),
# box_t2 (bt2), the plain six-face sequence (bplain)
CO="--scene cornell --width 600 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zna "ab:main||$CO;bt2||$CO;bplain||$CO;main||;bt2||;bplain||"
