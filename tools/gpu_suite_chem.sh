#!/bin/bash
# GPU job: the full GPU test suite, then the K12 kinetics benchmark (both kernels)
# and a PMC pass on the MFMA kernel.  Logs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/bench_chem.py --repeats 5 > gpurun_out/bench_chem.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_chem" -o run \
   -- python3 "$R/tools/bench_chem.py" --nx 1000 --ny 400 --repeats 2 > "$R/gpurun_out/pmc_chem.log" 2>&1)
