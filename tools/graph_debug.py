"""Step-graph vs eager debugging: steps both paths in windows and prints the
first divergence (dt, time, rho)."""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
import openhyperflow2d_amd as hf
from openhyperflow2d_amd.models import decks
text = decks.wedge15(300, 60, nmax=10 ** 6, nout=10 ** 5)
a = hf.Simulation(text, "gpu"); b = hf.Simulation(text, "gpu"); b.solver.use_graph = False
seq = [int(x) for x in sys.argv[1].split(',')] if len(sys.argv) > 1 else [40, 13, 61]
for n in seq:
    try:
        a.step(n, residual=False); b.step(n, residual=False)
    except Exception as e:
        print("fail", n, e); break
    ra, rb = a.field("rho"), b.field("rho")
    print(n, "graphs", a.solver.graph_launches, "dt", a.summary()["dt"], b.summary()["dt"], "time", a.summary()["time"], b.summary()["time"], "maxdiff", np.abs(ra - rb).max(), flush=True)
