"""Timing probe of the persistent window kernel (hf2d_lean_persist) against
the per-step tile kernel on the headline grid.  HF2D_PERSIST_DBG bits (debug
only; results are wrong with bits 1 and 8): 1 no grid barrier, 2 agent-scope
barrier atomics, 4 agent-scope dt atomics, 8 plain loads/stores for the
cross-tile border/halo traffic."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
os.environ.setdefault("HF2D_AUTOTUNE", "0")
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks  # noqa: E402


def timed(sim, n):
    try:
        sim.step(48)
    except RuntimeError:
        pass
    sim.solver.synchronize()
    t0 = time.perf_counter()
    try:   # debug variants may corrupt the state: keep the timing anyway
        sim.step(n)
    except RuntimeError:
        pass
    sim.solver.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


text = decks.wedge15(2000, 200, nmax=10 ** 6, nout=10 ** 5)
for window in [int(w) for w in (sys.argv[1:] or ["0", "6", "48", "192"])]:
    sim = hf.Simulation(text, "gpu", lean=True)
    sim.step(3)
    if window == 0:
        sim.solver.lean_persist = 0
    else:
        sim.solver.lean_persist = 1
        sim.solver.persist_steps = window
    us = timed(sim, int(os.environ.get("PROBE_STEPS", "480")))
    print("dbg=%s window %4d: %.2f us/step  launches=%d why=%r" % (os.environ.get("HF2D_PERSIST_DBG", "0"), window, us, sim.solver.persist_launches,
                                                          sim.solver.persist_why), flush=True)
