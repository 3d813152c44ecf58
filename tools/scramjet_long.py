#!/usr/bin/env python3
"""Long scramjet run in chunks: step, dt, T range, hot-cell share after each
chunk, to locate where a long run (bench.py --hot) leaves the stable range.

  python tools/scramjet_long.py --steps 30000 --chunk 2000 [--split]

--split runs the split predict / fill pair instead of the lean mechanism step.
A chunk that ends in the Tg < 0 error prints it and stops."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--split", action="store_true")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    if a.split:
        sim.solver.lean_mech = False
    tchem = sim.case.chem_tmin
    done = 0
    while done < a.steps:
        try:
            sim.step(a.chunk)
        except RuntimeError as e:
            print("after %d + <=%d steps: %s" % (done, a.chunk, e), flush=True)
            T = np.asarray(sim.field("T"))
            bad = np.argwhere(~(T > 0))
            print("cells with T <= 0 or nan: %d, first %s" % (len(bad), bad[:5].tolist()), flush=True)
            return 1
        done += a.chunk
        T = np.asarray(sim.field("T"))
        act = T[T > 0]
        print("step %6d dt %.4e  T %.1f .. %.1f  hot %.1f %%  lean steps %d" % (
            done, sim.summary()["dt"], act.min(), act.max(), 100 * (T >= tchem).mean(), sim.solver.lnm_steps),
            flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
