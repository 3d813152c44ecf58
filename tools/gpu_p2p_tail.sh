set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "p2p or virtual" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p2p.log 2>&1 && \
: > gpurun_out/p2p_tail.log && \
for nx in 2000 260; do
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx $nx --tail 10 --nofuse >> gpurun_out/p2p_tail.log 2>&1 || exit 1
done
