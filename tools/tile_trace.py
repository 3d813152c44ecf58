"""Phase timeline of one lean tile step from the in-kernel trace
(DeviceSolver.trace_tile: s_memrealtime at 100 MHz, per workgroup).

  python tools/tile_trace.py --nx 250 --ny 200 [--cpt 2 --tj 0]
Prints, in microseconds relative to the first workgroup's entry: the spread
of workgroup start times (dispatch ramp), the per-workgroup phase durations
(staging -> barrier, wave-0 compute, block reduction barrier, dt atomic) and
the end of the last workgroup, plus workgroups per CU / XCC (HW_ID, XCC_ID).
"""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def q(a, p):
    return float(np.percentile(a, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=250)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--cpt", type=int, default=0)
    ap.add_argument("--tj", type=int, default=-1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nt", type=int, default=256, help="threads per workgroup (256, 128, 64)")
    a = ap.parse_args()
    os.environ.setdefault("HF2D_AUTOTUNE", "0")
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.wedge15(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    s = sim.solver
    if a.cpt:
        s.lean_cpt = a.cpt
    if a.tj >= 0:
        s.lean_tj = a.tj
    s.lean_nt = a.nt
    print("grid %dx%d nt=%d cpt=%d tj=%d" % (a.nx, a.ny, s.lean_nt, s.lean_cpt, s.lean_tj))
    for rep in range(a.reps):
        t = np.asarray(s.trace_tile(20), dtype=np.uint64).reshape(-1, 8)
        t = t[t[:, 0] > 0]
        ts = t[:, :5].astype(np.int64)
        base = ts[:, 0].min()
        us = (ts - base) / 100.0   # 100 MHz ticks -> us
        hw = t[:, 5].astype(np.int64)
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        xcc = t[:, 6].astype(np.int64) & 0xF
        per_cu = collections.Counter(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
        per_xcc = collections.Counter(xcc.tolist())
        print("rep %d: %d workgroups on %d CUs (max %d per CU), per XCC %s" % (
            rep, len(t), len(per_cu), max(per_cu.values()), dict(sorted(per_xcc.items()))))
        print("  start      p0 %.2f  p50 %.2f  p90 %.2f  max %.2f" % (0.0, q(us[:, 0], 50), q(us[:, 0], 90), us[:, 0].max()))
        for k, name in ((1, "staged"), (2, "computed"), (3, "reduced"), (4, "atomic")):
            d = us[:, k] - us[:, k - 1]
            print("  %-9s  p10 %.2f  p50 %.2f  p90 %.2f  max %.2f" % (name, q(d, 10), q(d, 50), q(d, 90), d.max()))
        life = us[:, 4] - us[:, 0]
        print("  WG life    p10 %.2f  p50 %.2f  p90 %.2f  max %.2f" % (q(life, 10), q(life, 50), q(life, 90), life.max()))
        print("  last WG done at %.2f us after the first WG started" % us[:, 4].max())


if __name__ == "__main__":
    main()
