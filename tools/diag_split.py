#!/usr/bin/env python3
"""Diagnose a strip run that differs from one GPU: step the virtual ranks
(tests/test_gpu_kernels.py _virtual_ranks) and the one-GPU reference one
chunk at a time and print, per chunk, the columns where rho first differs.

  python tools/diag_split.py --deck scramjet --p2p fx --parts 0,97,194,214 --chunks 1x8,6x4"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--deck", default="scramjet")
    ap.add_argument("--p2p", default="fx")
    ap.add_argument("--parts", default="0,97,194,214")
    ap.add_argument("--chunks", default="1x8,6x4", help="NxK: K chunks of N plain steps")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from tests.test_gpu_kernels import _virtual_ranks

    cuts = [int(x) for x in a.parts.split(",")]
    parts = list(zip(cuts[:-1], cuts[1:]))
    nx = cuts[-1]
    text = (decks.resonator(nx, 40, nmax=10 ** 6, nout=10 ** 5) if a.deck == "resonator"
            else decks.scramjet(nx, 48, nmax=10 ** 6, nout=10 ** 5))
    sched = []
    for c in a.chunks.split(","):
        n, k = (int(x) for x in c.split("x"))
        sched += [(n, False)] * k
    ref = hf.Simulation(text, "gpu")
    for q in range(1, len(sched) + 1):
        got, summ = _virtual_ranks(hf, text, len(parts), sched[:q], lean=True, p2p=bool(a.p2p),
                                   fuse=a.p2p == "fx", parts=parts, fields=("rho", "T"))
        ref.step(sched[q - 1][0])
        d = np.abs(got["rho"] - np.asarray(ref.field("rho")))
        cols = sorted(set(np.nonzero(d.max(axis=1))[0].tolist()))
        print("after %d steps: dt %s vs %s, rho differs in %d columns %s" % (
            sum(n for n, _ in sched[:q]), summ["dt"], ref.summary()["dt"], len(cols), cols[:40]), flush=True)
        if cols:
            break


if __name__ == "__main__":
    main()
