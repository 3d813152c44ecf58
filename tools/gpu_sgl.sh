set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "single_gas or baseline or keps or graphs" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sgl.log 2>&1 ; \
timeout -k 10 120 python bench.py --config step --steps 200 --warmup 20 > gpurun_out/bench_step.log 2>&1 && \
timeout -k 10 120 python bench.py --config resonator --steps 200 --warmup 20 > gpurun_out/bench_resonator.log 2>&1
