# book-2 instances: box_t1f (near pass + six-face fallback, e1f) vs box_t2 (main); main now has box_t1f in
# the reference-scene instance
F="--scene final --width 1920 --aspect std16x9 --spp 200"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05z4a "ab:main||$F;e1f||$F"
