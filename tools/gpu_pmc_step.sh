set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && cd $R
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_scr -o f -- python3 bench.py --config scramjet --steps 20 --warmup 2 > gpurun_out/pmc_scr.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_scr -o w -- python3 bench.py --config scramjet --steps 20 --warmup 2 >> gpurun_out/pmc_scr.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_scr -o s -- python3 bench.py --config scramjet --steps 20 --warmup 2 >> gpurun_out/pmc_scr.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_scr -o scr -- python3 bench.py --config scramjet --steps 200 --warmup 20 > gpurun_out/prof_scr.log 2>&1
