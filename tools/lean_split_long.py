#!/usr/bin/env python3
"""Lean mechanism step vs the split pair over a long scramjet run: the same
deck stepped (a) lean in chunks with a download after each, (b) split in the
same chunks, (c) lean in one call; fields compared at the end (bitwise and
max relative difference), plus the first chunk where (a) and (b) differ.

  python tools/lean_split_long.py --steps 6000 --chunk 2000"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8)
    lean = hf.Simulation(text, "gpu")
    split = hf.Simulation(text, "gpu")
    split.solver.lean_mech = False
    fields = ["rho", "U", "V", "p", "T", "Y:H2", "Y:OH"]
    done = 0
    while done < a.steps:
        lean.step(a.chunk)
        split.step(a.chunk)
        done += a.chunk
        diffs = {}
        for f in fields:
            x, y = np.asarray(lean.field(f)), np.asarray(split.field(f))
            if not np.array_equal(x, y):
                d = np.abs(x - y)
                k = int(np.argmax(d))
                diffs[f] = (float(d.max() / max(np.abs(y).max(), 1e-300)), int((d > 0).sum()), np.unravel_index(k, x.shape))
        print("step %d: dt lean %r split %r; differing fields %s" % (
            done, lean.summary()["dt"], split.summary()["dt"], diffs or "none"), flush=True)
    one = hf.Simulation(text, "gpu")
    one.step(a.steps)
    for f in fields:
        x, y = np.asarray(one.field(f)), np.asarray(lean.field(f))
        print("one call vs chunked lean, %s: %s" % (f, "equal" if np.array_equal(x, y) else
                                                      "max rel diff %.3e" % (np.abs(x - y).max() / np.abs(y).max())),
              flush=True)


if __name__ == "__main__":
    main()
