#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for s in 0 100 200; do
  for c in resonator step; do
    HF2D_LNS_STAGGER=$s timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/lnsst_${c}_$s.log 2>&1 || exit 1
  done
done
bash tools/strip_proxy.sh
