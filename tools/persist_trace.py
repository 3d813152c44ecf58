"""Phase trace of the persistent window kernel (DeviceSolver.persist_trace):
per step, the p50 / p90 over workgroups of compute, commit, barrier wait and
halo-load times (us), and the spread of the step start."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
os.environ.setdefault("HF2D_AUTOTUNE", "0")
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks  # noqa: E402

nx, ny = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (2000, 200)))
sim = hf.Simulation(decks.wedge15(nx, ny, nmax=10 ** 6, nout=10 ** 5), "gpu", lean=True)
sim.solver.lean_persist = 1
sim.step(3)
tr = np.array(sim.solver.persist_trace(8), dtype=np.float64)
nt = sim.solver.persist_trace_tiles
tr = tr.reshape(nt, 8, 6)
t0 = tr[:, 0, 0].min()
print("tiles", nt, "XCDs", sorted(set(tr[:, 0, 5].astype(int) & 7)))
for s in range(7):
    st, cp, cm, br, hl = (tr[:, s, k] for k in range(5))
    q = lambda v: "%6.2f/%6.2f" % (np.percentile(v, 50) / 100.0, np.percentile(v, 90) / 100.0)  # noqa: E731
    print("step %d start+%7.2f (spread %5.2f)  compute %s  commit %s  barrier %s  halo %s" % (
        s, (st.min() - t0) / 100.0, (st.max() - st.min()) / 100.0, q(cp - st), q(cm - cp), q(br - cm), q(hl - br)))
