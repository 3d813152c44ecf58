#!/usr/bin/env python3
"""First step at which the lean mechanism step and the split pair differ on
the full scramjet (after --start steps in one call, equal there): bisects k in
(0, --span] with fresh runs of start + k steps, then prints the cells that
differ at the first differing k (fields, CT flags, local dt of both runs from
their downloaded state, and each run's dt-limiting cell).

  python tools/lean_split_bisect.py --start 2024 --span 24 [--download]"""
import argparse
import gc
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ["rho", "U", "V", "p", "T", "k", "R", "mu_t", "S7", "S8", "Y:H2", "Y:OH"]


def run(hf, text, start, k, dl):
    sims = []
    for lean in (True, False):
        s = hf.Simulation(text, "gpu")
        s.solver.lean_mech = lean
        s.step(start)
        if dl:
            s.solver.download()   # materialise the lean representation, re-enter on the next step
        s.step(k)
        s.solver.download()
        sims.append(s)
    out = []
    for s in sims:
        f = {n: np.asarray(s.case.field(n)).copy() for n in FIELDS + ["CT"]}
        f["dt"] = s.summary()["dt"]
        out.append(f)
    del sims
    gc.collect()
    return out


def local_dt(f, cfl, dx, dy):
    a = np.sqrt(np.maximum(f["k"] * f["R"] * f["T"], 0.0))
    with np.errstate(divide="ignore", invalid="ignore"):
        d = cfl * np.minimum(dx / (a + np.abs(f["U"])), dy / (a + np.abs(f["V"])))
    d[~np.isfinite(d)] = np.inf
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=2024)
    ap.add_argument("--span", type=int, default=24)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--download", action="store_true", help="download after the start call")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8)
    lo, hi = 0, a.span   # equal after start + lo, different after start + hi (checked)
    res = {}

    def differs(k):
        if k not in res:
            L, S = run(hf, text, a.start, k, a.download)
            d = L["dt"] != S["dt"] or any(not np.array_equal(L[n], S[n]) for n in FIELDS)
            res[k] = (d, L, S)
            print("k=%d: %s (dt %r vs %r)" % (k, "differ" if d else "equal", L["dt"], S["dt"]), flush=True)
        return res[k][0]

    if not differs(hi):
        print("no difference within %d steps" % hi, flush=True)
        return
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if differs(mid):
            hi = mid
        else:
            lo = mid
    _, L, S = res[hi]
    bad = np.zeros_like(L["rho"], dtype=bool)
    for n in FIELDS:
        d = L[n] != S[n]
        if d.any():
            print("  after start+%d: %s differs at %d cells" % (hi, n, int(d.sum())), flush=True)
        bad |= d
    cells = np.argwhere(bad)
    for i, j in cells[:16]:
        print("  cell (%d, %d) CT 0x%x T %r/%r rho %r/%r Y:H2 %r/%r" % (
            i, j, int(L["CT"][i, j]), L["T"][i, j], S["T"][i, j], L["rho"][i, j], S["rho"][i, j],
            L["Y:H2"][i, j], S["Y:H2"][i, j]), flush=True)
    if lo in res:
        _, L0, S0 = res[lo]
        case = hf.native().Case.from_deck(text, ".", False)
        cfl = 0.1
        dL = local_dt(L0, cfl, case.dx, case.dy)
        dS = local_dt(S0, cfl, case.dx, case.dy)
        for name, d in (("lean", dL), ("split", dS)):
            q = np.unravel_index(int(np.argmin(d)), d.shape)
            print("  %s state after start+%d: smallest local dt %r at %s" % (name, lo, float(d[q]), q), flush=True)


if __name__ == "__main__":
    main()
