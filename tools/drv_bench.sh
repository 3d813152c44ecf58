#!/bin/bash
# The driver's bench command (N=1), three times, one JSON line each.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_bench_$r.log 2>&1 || exit $?
  grep '^{' gpurun_out/drv_bench_$r.log
done
