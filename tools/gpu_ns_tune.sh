#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for c in resonator step; do
  timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 10 > gpurun_out/nst_$c.log 2>&1 || exit 1
done
