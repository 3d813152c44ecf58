set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
for c in step resonator triple_point scramjet; do
  timeout -k 10 240 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/bench_$c.log 2>&1 || exit 1
done
