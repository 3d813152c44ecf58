set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_chem_mech.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_chem.log 2>&1 && \
timeout -k 10 200 python tools/bench_chem.py > gpurun_out/bench_chem.log 2>&1 && \
timeout -k 10 200 python tools/bench_chem.py --nsub 1 > gpurun_out/bench_chem_nsub1.log 2>&1
