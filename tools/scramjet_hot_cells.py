"""Share of scramjet cells (and of 64-cell wavefronts) above the kinetics
threshold Tchem: how much of hf2d_chem_fast's grid does work."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks  # noqa: E402

sim = hf.Simulation(decks.scramjet(6000, 400, nmax=10 ** 9, nout=10 ** 8), "gpu")
for n in (0, 200, 1000):
    if n:
        sim.step(n)
    T = np.asarray(sim.field("T")).reshape(-1)   # x-major: cell index i*ny + j
    hot = T >= 600.0
    w = hot[: len(hot) // 64 * 64].reshape(-1, 64).any(axis=1)
    print("after %5d more steps: hot cells %.1f %%, wavefronts with a hot cell %.1f %%" % (
        n, 100 * hot.mean(), 100 * w.mean()), flush=True)
