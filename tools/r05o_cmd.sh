# final_scene after flattening: 768-thread (3 waves) vs 1024-thread (4 waves) book-2 block; phase clocks
F="--scene final --width 1920 --aspect std16x9 --spp 200" &&
AB_STEPS=3 AB_REPS=2 bash tools/gpu.sh r05o1 "ab:main||$F;main|SHIRLEY_WIDE4=1|$F" &&
bash tools/gpu.sh r05o2 "sh:SHIRLEY_LIB_DIR=$PWD/exp/phase python bench.py --steps 1 --warmup 1 --no-cpu --no-configs $F" &&
bash tools/gpu.sh r05o3 "sh:SHIRLEY_LIB_DIR=$PWD/exp/phase python bench.py --steps 1 --warmup 1 --no-cpu --no-configs --scene spheres --width 1920 --aspect std16x9 --spp 200" &&
GS="--scene spheres --width 1920 --aspect std16x9 --spp 200" &&
AB_STEPS=10 AB_REPS=2 bash tools/gpu.sh r05o4 "ab:main||$GS;main|SHIRLEY_LDS_NODES=64|$GS;main|SHIRLEY_LDS_NODES=128|$GS"
