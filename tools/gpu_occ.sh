set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/occ_sweep.py > gpurun_out/occ_sweep.log 2>&1 && \
timeout -k 10 100 python tools/occ_sweep.py --nx 250 --wgcu 0,2,1 >> gpurun_out/occ_sweep.log 2>&1
