set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 500 --warmup 50 > $R/gpurun_out/prof_bench.log 2>&1
