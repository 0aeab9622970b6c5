# round 5 end: the final build's evidence — GPU suite, smoke, the full bench line (configs + CPU baseline),
# headline kernel stats + HBM traffic + VALU + wait states, and the book-2 final_scene (cfg5) profile
V="SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_THREAD_CYCLES_VALU,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_SALU"
W1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_SMEM,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS"
W2="SQ_WAVE_CYCLES,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_BUSY_CYCLES"
C5="--scene final --width 1920 --aspect std16x9 --spp 2000"
ONE="--steps 1 --warmup 0 --no-cpu --no-configs"
bash tools/gpu.sh r05z tests smoke bench &&
bash tools/gpu.sh r05z_head prof "pmc:FETCH_SIZE" "pmc:WRITE_SIZE" "pmc:$V:$ONE" "pmc:$W1:$ONE" "pmc:$W2:$ONE" &&
bash tools/gpu.sh r05z_cfg5 "prof:--steps 2 --warmup 1 --no-cpu --no-configs $C5" "pmc:FETCH_SIZE:$ONE $C5" "pmc:WRITE_SIZE:$ONE $C5" "pmc:$V:$ONE $C5"
