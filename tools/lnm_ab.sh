#!/bin/bash
# timing-only A/B of lean-mech phases
cd ${GRAFT_REPO_ROOT:-.}
for d in 0 1 2 4 7; do
  HF2D_LNM_DBG=$d timeout -k 10 120 python bench.py --config scramjet --steps 60 --warmup 10 > gpurun_out/lnm_dbg_$d.log 2>&1 || exit 1
done
