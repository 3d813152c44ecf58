# Strip-size sweep: standalone strip bench with / without autotune, and the
# 2-rank tail proxy (rank 0 = 250 columns) with the exchange kernel.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/strips.log
for nx in 250 500 1000; do
  timeout -k 10 120 python bench.py --nx $nx --steps 3000 --warmup 300 >> gpurun_out/strips.log 2>&1 || exit 1
  HF2D_AUTOTUNE=0 timeout -k 10 120 python bench.py --nx $nx --steps 3000 --warmup 300 >> gpurun_out/strips.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx 260 --tail 10 --nofuse --steps 3000 --warmup 300 >> gpurun_out/strips.log 2>&1 && \
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx 260 --tail 10 --nofuse --autotune --steps 3000 --warmup 300 >> gpurun_out/strips.log 2>&1 && \
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx 260 --tail 10 --autotune --steps 3000 --warmup 300 >> gpurun_out/strips.log 2>&1
