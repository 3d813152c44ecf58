set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && cd $R
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_bw -o f -- python3 tools/bw_calibrate.py 80 > gpurun_out/pmc_bw.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_bw -o w -- python3 tools/bw_calibrate.py 80 >> gpurun_out/pmc_bw.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lean -o f -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/pmc_lean.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_lean -o w -- python3 bench.py --steps 20 --warmup 2 >> gpurun_out/pmc_lean.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_lean -o s -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/pmc_lean2.log 2>&1
