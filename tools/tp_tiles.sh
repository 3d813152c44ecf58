#!/bin/bash
# triple point under fixed tile geometries (1 GPU)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config triple_point --steps 100 --warmup 10 > gpurun_out/tp_auto.log 2>&1 || exit 1
for t in ${TILES:-1,50 2,0 2,64 1,0}; do
  timeout -k 10 200 python bench.py --config triple_point --steps 100 --warmup 10 --tile $t > gpurun_out/tp_$t.log 2>&1 || exit 1
done
