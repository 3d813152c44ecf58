"""K12 MFMA mechanism chemistry benchmark: one chemistry call on a scramjet-sized
field (6000x400 = 2.4 M cells, demo 8-species / 12-step H2-air mechanism), checked on
a cell subset against the PyTorch FP64 reference.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openhyperflow2d_amd.ops import chemistry as ch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--nsub", type=int, default=4)
    ap.add_argument("--dt", type=float, default=1e-7)
    ap.add_argument("--repeats", type=int, default=10)
    a = ap.parse_args()
    m = ch.h2_air_demo()
    n = a.nx * a.ny
    Y, T = ch.demo_state(m, n, seed=11)
    got, ms = ch.mech_step_gpu(m, Y, T, a.dt, a.nsub, repeats=a.repeats)
    sel = np.random.default_rng(0).choice(n, size=min(n, 4096), replace=False)
    ref = ch.reference_step(m, Y[:, sel], T[sel], a.dt, a.nsub)
    err = float(np.abs(got[:, sel] - ref).max() / np.abs(ref).max())
    R = m.packed()[0].shape[1]
    # MFMA work actually issued: per 16-cell tile and substep, (1 + 16) chains of R/4 16x16x4 f64 MFMAs
    mfma_flop = (n / 16) * a.nsub * 17 * (R / 4) * (2 * 16 * 16 * 4)
    print(json.dumps({"metric": "K12 mechanism chemistry", "cells": n, "species": m.ns, "reactions": len(m.reactions),
                      "nsub": a.nsub, "ms_per_call": ms, "Mcells_per_s": n / ms / 1e3,
                      "mfma_f64_tflops": mfma_flop / ms / 1e9, "rel_err_vs_torch_fp64": err}))
    if not err < 1e-10:
        raise SystemExit("mismatch vs reference: %g" % err)


if __name__ == "__main__":
    main()
