# round 5: wait-state passes on the headline, cfg4 / cfg5 kernel stats + traffic + VALU, gloo rehearsal
V="SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_THREAD_CYCLES_VALU,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_SALU"
C4="--scene cornell --width 600 --aspect square --spp 10000"
C5="--scene final --width 1920 --aspect std16x9 --spp 2000"
ONE="--steps 1 --warmup 0 --no-cpu --no-configs"
bash tools/gpu.sh r05e_waits "pmc:SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_SMEM,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS:$ONE" "pmc:SQ_WAVE_CYCLES,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_BUSY_CYCLES:$ONE" &&
bash tools/gpu.sh r05e_cfg4 "prof:--steps 2 --warmup 1 --no-cpu --no-configs $C4" "pmc:FETCH_SIZE:$ONE $C4" "pmc:WRITE_SIZE:$ONE $C4" "pmc:$V:$ONE $C4" &&
bash tools/gpu.sh r05e_cfg5 "prof:--steps 2 --warmup 1 --no-cpu --no-configs $C5" "pmc:FETCH_SIZE:$ONE $C5" "pmc:WRITE_SIZE:$ONE $C5" "pmc:$V:$ONE $C5" &&
# (then the phase clocks of the book-2 final scene, the headline and Cornell: instrumented build exp/phase)
bash tools/rehearsal.sh gpurun_out/r05e_reh &&
bash tools/gpu.sh r05e_phase "sh:SHIRLEY_LIB_DIR=$PWD/exp/phase python bench.py --steps 1 --warmup 1 --no-cpu --no-configs --scene final --width 1920 --aspect std16x9 --spp 200" "sh:SHIRLEY_LIB_DIR=$PWD/exp/phase python bench.py --steps 1 --warmup 1 --no-cpu --no-configs" "sh:SHIRLEY_LIB_DIR=$PWD/exp/phase python bench.py --steps 1 --warmup 1 --no-cpu --no-configs --scene cornell --width 600 --aspect square --spp 1000"
