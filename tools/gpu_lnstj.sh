#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for tj in 0 16 20 25 40 50; do
  timeout -k 10 200 python bench.py --config resonator --steps 200 --warmup 10 --tile 1,$tj > gpurun_out/tj_reso_$tj.log 2>&1 || exit 1
done
for tj in 0 16 25 40; do
  timeout -k 10 200 python bench.py --config step --steps 200 --warmup 10 --tile 1,$tj > gpurun_out/tj_step_$tj.log 2>&1 || exit 1
done
