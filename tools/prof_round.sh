#!/bin/bash
# Round profile on one GPU box: rocprofv3 kernel-trace stats of the headline
# (autotune off, the autotune's usual pick fixed, so no candidate runs land in
# the table) and of the resonator / scramjet configs, plus PMC passes of the
# headline tile kernel.  Every step has its own time limit; the first failure
# ends the script.
#   bash tools/prof_round.sh OUTDIR [TILE]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/prof}
T=${2:-1,16,64}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
stats() {   # tag, bench args...
  local tag=$1; shift
  HF2D_AUTOTUNE=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$tag" -o run -- \
    python3 "$R/bench.py" "$@" > "$O/$tag.log" 2>&1
}
pmc() {   # tag, counters...
  local tag=$1; shift
  HF2D_AUTOTUNE=0 timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$O/$tag" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 2 --tile "$T" > "$O/$tag.log" 2>&1
}
stats headline --steps 200 --warmup 20 --tile "$T" &&
stats resonator --config resonator --steps 100 --warmup 10 &&
stats scramjet --config scramjet --steps 20 --warmup 3 &&
pmc p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
pmc p2 FETCH_SIZE TCC_HIT_sum &&
pmc p3 WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE &&
pmc p4 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES
