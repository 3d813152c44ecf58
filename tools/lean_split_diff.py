#!/usr/bin/env python3
"""Locate the first cells where the lean mechanism step and the split pair
part ways on the full scramjet: both advance --start steps, then --every
steps at a time until some field differs; prints the differing cells with
their CT flags and the fields that differ there.

  python tools/lean_split_diff.py --start 2000 --every 6 --max 2400 [--pair lean-lean]

--pair lean-lean / split-split runs the same path twice (a determinism check).
(The names `lean` / `split` below are the first / second run of the pair.)"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ["rho", "U", "V", "p", "T", "k", "mu_t", "mu", "S7", "S8", "Y:H2", "Y:OH"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=2000)
    ap.add_argument("--every", type=int, default=6)
    ap.add_argument("--max", type=int, default=2400)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--pair", default="lean-split", choices=["lean-split", "lean-lean", "split-split"])
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8)
    lean = hf.Simulation(text, "gpu")
    split = hf.Simulation(text, "gpu")
    first, second = a.pair.split("-")
    lean.solver.lean_mech = first == "lean"
    split.solver.lean_mech = second == "lean"
    print("pair %s" % a.pair, flush=True)
    lean.step(a.start)
    split.step(a.start)
    done = a.start
    reports = 0
    while done < a.max and reports < 3:
        lean.step(a.every)
        split.step(a.every)
        done += a.every
        bad = None
        which = {}
        lean.solver.download()   # (Simulation.field downloads the whole record per call)
        split.solver.download()
        fl = {f: np.asarray(lean.case.field(f)) for f in FIELDS + ["CT"]}
        fs = {f: np.asarray(split.case.field(f)) for f in FIELDS}
        for f in FIELDS:
            x, y = fl[f], fs[f]
            d = x != y
            if d.any():
                which[f] = int(d.sum())
                bad = d if bad is None else (bad | d)
        if bad is None:
            print("step %d: equal" % done, flush=True)
            continue
        reports += 1
        ct = fl["CT"]
        cells = np.argwhere(bad)
        print("step %d: %d cells differ; per field %s; dt %r vs %r" % (
            done, len(cells), which, lean.summary()["dt"], split.summary()["dt"]), flush=True)
        for i, j in cells[:12]:
            vals = {f: (float(fl[f][i, j]), float(fs[f][i, j])) for f in ("T", "rho", "mu_t", "Y:H2")}
            print("  cell (%d, %d) CT 0x%x %s" % (i, j, int(ct[i, j]), vals), flush=True)
        cols = np.unique(cells[:, 0])
        print("  columns %s .. %s, rows %s .. %s" % (cols.min(), cols.max(), cells[:, 1].min(), cells[:, 1].max()),
              flush=True)
    if reports == 0:
        print("no difference up to step %d" % done, flush=True)


if __name__ == "__main__":
    main()
