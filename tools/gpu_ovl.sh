#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "strip or virtual or p2p or overlap or lean_ns" > gpurun_out/pytest_ovl.log 2>&1 &&
for c in step resonator scramjet; do
  timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/ovl_$c.log 2>&1 || exit 1
done
