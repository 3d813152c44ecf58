#!/bin/bash
# PMC passes (one rocprofv3 run each) of the headline bench at a fixed tile geometry:
#   TILE=cpt,tj,nt bash tools/pmc_tile.sh   -> gpurun_out/r4e/p*/ ; summary: tools/pmc_summary.py
mkdir -p gpurun_out/r4e && cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
T=${TILE:-1,8,128}
run() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/r4e/$tag -o run -- python3 $R/bench.py --steps 20 --warmup 2 --tile $T > $R/gpurun_out/r4e/$tag.log 2>&1; }
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
run p2 FETCH_SIZE TCC_HIT_sum && run p3 WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE && \
run p4 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES && \
run p5 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT
