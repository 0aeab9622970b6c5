# node order in memory: breadth-first (main) vs depth-first over sibling groups (SHIRLEY_NODE_DFS)
S="--scene spheres --width 1920 --aspect std16x9 --spp 200"
F="--scene final --width 1920 --aspect std16x9 --spp 200"
CO="--scene cornell --width 600 --aspect square --spp 1000"
AB_STEPS=3 AB_REPS=3 bash tools/gpu.sh r05zma "ab:main||$S;main|SHIRLEY_NODE_DFS=1|$S;main||$F;main|SHIRLEY_NODE_DFS=1|$F;main||;main|SHIRLEY_NODE_DFS=1|;main||$CO;main|SHIRLEY_NODE_DFS=1|$CO" &&
SHIRLEY_NODE_DFS=1 bash tools/gpu.sh r05zmc "tests:tests/test_gpu_parity.py -k collapse_choice or render_matches"
