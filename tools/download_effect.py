#!/usr/bin/env python3
"""Does a mid-run download change the trajectory?  Runs a deck on one GPU
continuously and again with Simulation.field() (download + materialise)
after every step, and prints where dt / rho first differ.

  python tools/download_effect.py --deck scramjet --steps 8"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--deck", default="scramjet")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--nx", type=int, default=214)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    gen = {"scramjet": lambda: decks.scramjet(a.nx, 48, nmax=10 ** 6, nout=10 ** 5),
           "resonator": lambda: decks.resonator(a.nx, 40, nmax=10 ** 6, nout=10 ** 5),
           "step": lambda: decks.step(a.nx, 80, nmax=10 ** 6, nout=10 ** 5)}[a.deck]
    cont = hf.Simulation(gen(), "gpu")
    down = hf.Simulation(gen(), "gpu")
    for s in range(1, a.steps + 1):
        cont.step(1)
        down.step(1)
        down.field("rho")
        # compare without downloading `cont` mid-run: its summary only
        print("step %d: dt continuous %r  with downloads %r" % (s, cont.summary()["dt"], down.summary()["dt"]),
              flush=True)
    r1, r2 = np.asarray(cont.field("rho")), np.asarray(down.field("rho"))
    print("rho equal at the end:", bool(np.array_equal(r1, r2)), "max diff", float(np.abs(r1 - r2).max()))


if __name__ == "__main__":
    main()
