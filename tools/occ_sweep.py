"""Lean tile geometry x residency sweep on one GPU: us/step for cells per
thread (cpt), tile height (tj) and resident workgroups per CU (wgcu, forced
through the LDS request; 0 = as many as fit).

  python tools/occ_sweep.py --nx 2000 --ny 200
"""
import argparse
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--cpt", default="1,2")
    ap.add_argument("--tj", default="0,16,32")
    ap.add_argument("--wgcu", default="0,3,2,1")
    a = ap.parse_args()
    os.environ.setdefault("HF2D_AUTOTUNE", "0")
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.wedge15(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    s = sim.solver
    sim.step(50)
    ints = lambda t: [int(x) for x in t.split(",")]
    rows = []
    for cpt, tj, wg in itertools.product(ints(a.cpt), ints(a.tj), ints(a.wgcu)):
        s.lean_cpt, s.lean_tj, s.lean_wgcu = cpt, tj, wg
        try:
            sim.step(30)
            s.synchronize()
            best = 1e30
            for _ in range(2):
                t0 = time.perf_counter()
                sim.step(a.steps)
                s.synchronize()
                best = min(best, (time.perf_counter() - t0) / a.steps * 1e6)
        except RuntimeError as e:
            print("cpt=%d tj=%d wgcu=%d failed: %s" % (cpt, tj, wg, e), flush=True)
            continue
        rows.append((best, cpt, tj, wg))
        print("cpt=%d tj=%2d wgcu=%d  %.2f us/step" % (cpt, tj, wg, best), flush=True)
    rows.sort()
    print("best: cpt=%d tj=%d wgcu=%d %.2f us/step" % (rows[0][1], rows[0][2], rows[0][3], rows[0][0]))


if __name__ == "__main__":
    main()
