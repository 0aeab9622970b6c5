# Cornell @ 10k: vector-memory instruction counts and writes with the optimal (auto) and the greedy tree
C4="--scene cornell --width 600 --aspect square --spp 10000"
ONE="--steps 1 --warmup 0 --no-cpu --no-configs"
bash tools/gpu.sh r05zl_dp "pmc:SQ_WAVE_CYCLES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS:$ONE $C4" "pmc:WRITE_SIZE:$ONE $C4" &&
SHIRLEY_COLLAPSE_DP=0 bash tools/gpu.sh r05zl_gr "pmc:SQ_WAVE_CYCLES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS:$ONE $C4" "pmc:WRITE_SIZE:$ONE $C4"
