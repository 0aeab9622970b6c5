# cfg4 (Cornell @ 10 000 spp) kernel stats, HBM traffic and VALU on the collapse-choice kernel
V="SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_THREAD_CYCLES_VALU,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_SALU"
C4="--scene cornell --width 600 --aspect square --spp 10000"
ONE="--steps 1 --warmup 0 --no-cpu --no-configs"
bash tools/gpu.sh r05zk_cfg4 "prof:--steps 2 --warmup 1 --no-cpu --no-configs $C4" "pmc:FETCH_SIZE:$ONE $C4" "pmc:WRITE_SIZE:$ONE $C4" "pmc:$V:$ONE $C4"
