set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/p2p_tail.log
for nx in 2000 260; do
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx $nx --tail 10 >> gpurun_out/p2p_tail.log 2>&1 && \
timeout -k 10 120 python tools/p2p_probe.py --ranks 2 --nx $nx --tail 10 --nofuse >> gpurun_out/p2p_tail.log 2>&1 && \
timeout -k 10 120 python bench.py --nx $((nx-10)) --ny 200 --steps 600 --warmup 60 >> gpurun_out/p2p_tail.log 2>&1 || exit 1
done
