set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_at.log 2>&1 && \
timeout -k 10 200 python -c "
import time
import openhyperflow2d_amd as hf
from openhyperflow2d_amd.models import decks
for name, t in (('wedge', decks.wedge15(2000, 200, nmax=10**9, nout=10**8)), ('tp', decks.triple_point(4000, 1000, nmax=10**9, nout=10**8))):
    t0 = time.time(); s = hf.Simulation(t, 'gpu'); print(name, '%.1f s' % (time.time() - t0), s.autotune_log[-60:], flush=True)
" > gpurun_out/autotune.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_at.log 2>&1 && \
timeout -k 10 200 python bench.py --config triple_point --steps 100 --warmup 10 >> gpurun_out/bench_at.log 2>&1
