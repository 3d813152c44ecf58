set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o full -- python bench.py --steps 600 --warmup 60 > gpurun_out/prof_b1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o strip250 -- python bench.py --nx 250 --ny 200 --steps 600 --warmup 60 > gpurun_out/prof_b2.log 2>&1
