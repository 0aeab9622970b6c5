# tree builder variants on the scene-in-LDS scenes (with the optimal collapse): SAH sweep (main), binned
# SAH, the reference's own tree
CO="--scene cornell --width 600 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05zia "ab:main||$CO;main|SHIRLEY_SAH_BINNED=1|$CO;main||$CO --bvh reference;main||;main|SHIRLEY_SAH_BINNED=1|;main||--bvh reference"
