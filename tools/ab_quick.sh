#!/bin/bash
# Quick 1-GPU measurements: config benches + headline under HF2D_STAGGER values
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in ${CONFIGS:-step resonator scramjet}; do
  st=100; [ $c = scramjet ] && st=40
  timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 > gpurun_out/q_$c.log 2>&1 || exit 1
done
for s in ${STAGGERS:-0 100 200 300}; do
  HF2D_STAGGER=$s HF2D_AUTOTUNE=0 timeout -k 10 120 python bench.py --steps 2000 --warmup 100 > gpurun_out/q_stag$s.log 2>&1 || exit 1
done
