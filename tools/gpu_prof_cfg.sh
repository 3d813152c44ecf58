# usage: bash tools/gpu_prof_cfg.sh <config> [more configs...]: kernel trace + HBM bytes per kernel
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && cd $R
for c in "$@"; do
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$c -o f -- python3 bench.py --config $c --steps 20 --warmup 2 > gpurun_out/pmc_$c.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_$c -o w -- python3 bench.py --config $c --steps 20 --warmup 2 >> gpurun_out/pmc_$c.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/pmc_$c -o s -- python3 bench.py --config $c --steps 20 --warmup 2 >> gpurun_out/pmc_$c.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o k -- python3 bench.py --config $c --steps 200 --warmup 20 > gpurun_out/prof_$c.log 2>&1 || exit 1
done
