set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1 ; \
timeout -k 10 200 python tools/ab_bench.py --variants tile,cpt1,march2 --steps 400 --rounds 3 > gpurun_out/ab_full.log 2>&1 && \
timeout -k 10 200 python tools/ab_bench.py --nx 250 --variants tile,march1 --steps 400 --rounds 3 > gpurun_out/ab_250.log 2>&1
