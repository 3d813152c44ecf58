#!/usr/bin/env python3
"""Host-side cost of a run_steps call on the GPU: step graphs vs eager
launches, on a grid small enough that the kernels take a few us, and the
headline grid with the driver's call shape (sync, 20 steps, sync).

  python tools/launch_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(sim, n, reps):
    sim.solver.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        sim.step(n)
        sim.solver.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e6


def main():
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    for nx, ny in ((200, 40), (2000, 200)):
        for graph in (True, False):
            sim = hf.Simulation(decks.wedge15(nx, ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
            sim.solver.use_graph = graph
            sim.step(48)
            for n in (1, 6, 20, 60):
                us = timed(sim, n, 20)
                print("%dx%d graphs=%d call of %2d steps: %8.1f us  (%6.2f us/step)" % (nx, ny, graph, n, us, us / n),
                      flush=True)


if __name__ == "__main__":
    main()
