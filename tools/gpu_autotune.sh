set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_at.log 2>&1 && \
timeout -k 10 120 python -c "
import openhyperflow2d_amd as hf
from openhyperflow2d_amd.models import decks
for nx in (2000, 250):
    s = hf.Simulation(decks.wedge15(nx, 200, nmax=10**9, nout=10**8), 'gpu')
    print(nx, s.autotune_log, flush=True)
" > gpurun_out/autotune.log 2>&1 && \
for r in 1 2; do timeout -k 10 120 python bench.py --steps 2000 --warmup 200 >> gpurun_out/bench_at.log 2>&1 || exit 1; done
