#!/usr/bin/env python3
"""Which stored quantities differ between the lean mechanism step and the
split pair after a download + re-entry: both runs step --start steps, download,
step --k more, and their full cell records (every CellRecord member) and
species are compared member by member.

  python tools/lean_split_records.py --start 2024 --k 10"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NEQ, NSPEC = 9, 4
REC = np.dtype([
    ("S", "f8", NEQ), ("dSdx", "f8", NEQ), ("dSdy", "f8", NEQ), ("TurbType", "u8"),
    ("l_min", "f8"), ("y_plus", "f8"), ("Re_local", "f8"), ("mu_t", "f8"), ("lam_t", "f8"),
    ("dkdx", "f8"), ("dkdy", "f8"), ("depsdx", "f8"), ("depsdy", "f8"), ("x", "f8"), ("y", "f8"),
    ("ix", "i4"), ("iy", "i4"), ("nb_ptr", "u8", 4), ("p", "f8"), ("idXl", "i4"), ("idYu", "i4"),
    ("idXr", "i4"), ("idYd", "i4"), ("NGX", "i4"), ("NGY", "i4"), ("CT", "u8"), ("i_wall", "i4"),
    ("j_wall", "i4"), ("beta", "f8", NEQ), ("Q_conv", "f8"), ("time", "f8"), ("k", "f8"), ("R", "f8"),
    ("lam", "f8"), ("mu", "f8"), ("CP", "f8"), ("Diff", "f8"), ("Tf", "f8"), ("A", "f8", NEQ),
    ("B", "f8", NEQ), ("F", "f8", NEQ), ("RX", "f8", NEQ), ("RY", "f8", NEQ), ("Src", "f8", NEQ),
    ("SrcAdd", "f8", NEQ), ("Tg", "f8"), ("U", "f8"), ("V", "f8"), ("Y", "f8", NSPEC), ("Uw", "f8"),
    ("Vw", "f8"), ("droYdx", "f8", NSPEC), ("droYdy", "f8", NSPEC), ("dUdx", "f8"), ("dUdy", "f8"),
    ("dVdx", "f8"), ("dVdy", "f8"), ("dTdx", "f8"), ("dTdy", "f8"), ("BGX", "f8"), ("BGY", "f8")])
assert REC.itemsize == 1248, REC.itemsize


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=2024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--nodl", action="store_true", help="no download after the start call")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.scramjet(6000, 400, nmax=10 ** 9, nout=10 ** 8)
    recs, sp = [], []
    for lean in (True, False):
        s = hf.Simulation(text, "gpu")
        s.solver.lean_mech = lean
        s.step(a.start)
        if not a.nodl:
            s.solver.download()
        s.step(a.k)
        r = np.frombuffer(s.records(), dtype=REC).copy()
        recs.append(r)
        sp.append({n: np.asarray(s.case.field("Y:" + n)).copy() for n in ("H2", "O2", "H", "O", "OH", "H2O", "HO2", "H2O2")})
        print("%s: dt %r" % ("lean" if lean else "split", s.summary()["dt"]), flush=True)
        del s
    L, S = recs
    nx, ny = 6000, 400
    for name in REC.names:
        x, y = L[name], S[name]
        if x.dtype.kind == "f":
            d = ~((x == y) | (np.isnan(x) & np.isnan(y)))
        else:
            d = x != y
        if d.ndim > 1:
            for c in range(d.shape[1]):
                if d[:, c].any():
                    cells = np.flatnonzero(d[:, c])
                    print("%s[%d]: %d cells differ, first (i, j) %s" % (name, c, len(cells),
                                                                  [(int(q // ny), int(q % ny)) for q in cells[:6]]),
                          flush=True)
        elif d.any():
            cells = np.flatnonzero(d)
            print("%s: %d cells differ, first (i, j) %s" % (name, len(cells), [(int(q // ny), int(q % ny)) for q in cells[:6]]),
                  flush=True)
    for n in sp[0]:
        d = sp[0][n] != sp[1][n]
        if d.any():
            q = np.argwhere(d)
            print("Y:%s: %d cells differ, first %s" % (n, len(q), q[:6].tolist()), flush=True)


if __name__ == "__main__":
    main()
