#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for o in 2 3 5; do
  timeout -k 10 200 python bench.py --config resonator --steps 200 --warmup 10 --lns-occ $o > gpurun_out/occ_reso_$o.log 2>&1 || exit 1
done
for o in 2 3; do
  timeout -k 10 200 python bench.py --config step --steps 200 --warmup 10 --lns-occ $o > gpurun_out/occ_step_$o.log 2>&1 || exit 1
done
