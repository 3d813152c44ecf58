set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "monitor or rccl" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mon.log 2>&1
