#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mechanism.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "lean_mech or lean_ns_strips or mech" > gpurun_out/pytest_lnm2.log 2>&1 &&
timeout -k 10 200 python bench.py --config scramjet --steps 100 --warmup 10 > gpurun_out/lnm2_scram.log 2>&1
