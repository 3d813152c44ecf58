# Fused (tail-wait) exchange vs the separate exchange kernel on the one-GPU
# proxy: bitwise p2p tests, then the --tail probe (rank 1 owns 10 columns).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "p2p or virtual" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fx.log 2>&1 && \
: > gpurun_out/fx_tail.log && \
for nx in 2000 260; do
  echo "nx=$nx separate" >> gpurun_out/fx_tail.log
  timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx $nx --tail 10 --nofuse --steps 3000 --warmup 300 >> gpurun_out/fx_tail.log 2>&1 || exit 1
  echo "nx=$nx fused" >> gpurun_out/fx_tail.log
  timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx $nx --tail 10 --steps 3000 --warmup 300 >> gpurun_out/fx_tail.log 2>&1 || exit 1
done
