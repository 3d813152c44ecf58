set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_bench.py --variants tile,cpt1 --steps 400 --rounds 4 > gpurun_out/ab_full.log 2>&1 && \
timeout -k 10 200 python tools/ab_bench.py --nx 250 --variants tile,cpt1 --steps 400 --rounds 4 > gpurun_out/ab_250.log 2>&1
