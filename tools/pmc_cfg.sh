#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) of bench.py ARGS, e.g.
#   bash tools/pmc_cfg.sh TAG --config step --steps 20 --warmup 2
# -> gpurun_out/pmc_TAG_{1..4}/run_counter_collection.csv (tools/pmc_summary.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1
shift
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
pass() {
  local n=$1
  shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_${tag}_$n" -o run \
    -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${tag}_$n.log" 2>&1
}
ARGS="$*"
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
pass 2 FETCH_SIZE TCC_HIT_sum &&
pass 3 WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE &&
pass 4 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES
