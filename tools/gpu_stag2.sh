#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for s in ${STAGS:-150 -150 -200 -250 -300}; do
  HF2D_STAGGER=$s timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --tile 2,20 > gpurun_out/st2_$s.log 2>&1 || exit 1
done
for c in ${CFGS:-triple_point step}; do
  timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/st2_$c.log 2>&1 || exit 1
done
