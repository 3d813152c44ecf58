set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_chem_mech.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_chem.log 2>&1 && \
timeout -k 10 200 python tools/bench_chem.py > gpurun_out/bench_chem.log 2>&1 && \
timeout -k 10 200 python tools/bench_chem.py --nsub 1 > gpurun_out/bench_chem_nsub1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_chem -o run -- python3 $R/tools/bench_chem.py --repeats 3 > $R/gpurun_out/prof_chem.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_chem -o run -- python3 $R/tools/bench_chem.py --repeats 2 > $R/gpurun_out/pmc_chem.log 2>&1
