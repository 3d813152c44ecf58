#!/usr/bin/env python3
"""Device time of the lean mechanism step's phases (tile kernel, kinetics of
the listed cells, state kernel of the reacting cells) on the scramjet, after N
untimed steps (the developed state: --hot 80000 is one flow-through), with
hipEvents around each phase (DeviceSolver.lnm_timing; no profiler needed).

  python tools/scramjet_phases.py --hot 80000 --steps 100"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hot", type=int, default=80000)
    ap.add_argument("--chunk", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    t0 = time.time()
    done = 0
    while done < a.hot:   # (progress lines: a silent GPU command looks hung)
        n = min(a.chunk, a.hot - done)
        sim.step(n)
        done += n
        print("hot steps %d (%.0f s)" % (done, time.time() - t0), flush=True)
    sim.solver.synchronize()
    T = np.asarray(sim.field("T"))
    hot = float((T >= sim.case.chem_tmin).mean())
    sim.solver.synchronize()
    t1 = time.perf_counter()
    sim.step(a.steps)
    sim.solver.synchronize()
    wall = (time.perf_counter() - t1) / a.steps * 1e3
    sim.solver.lnm_phase_ms = [0, 0, 0, 0]
    sim.solver.use_graph = False   # (every timed step through the host launch path)
    sim.solver.lnm_timing = True
    sim.step(a.steps)
    sim.solver.lnm_timing = False
    tile, chem, hotk, n = sim.solver.lnm_phase_ms
    rec = {"hot_steps": a.hot, "hot_share": round(hot, 4), "steps": int(n), "ms_per_step_untimed_run": round(wall, 4),
           "tile_ms": round(tile / n, 4), "kinetics_ms": round(chem / n, 4), "state_ms": round(hotk / n, 4),
           "kinetics_share": round(chem / (tile + chem + hotk), 4),
           "reacting_share": round((chem + hotk) / (tile + chem + hotk), 4)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
