#!/bin/bash
# strip / p2p GPU tests + the one-GPU strip proxies
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "strip or virtual or p2p or overlap" > gpurun_out/pytest_strips.log 2>&1 && bash tools/strip_proxy.sh
