#!/usr/bin/env python3
"""Long scramjet run in chunks: step, dt, T range, hot-cell share after each
chunk, and where the coldest cells sit (to locate a flow feature that leaves
the stable range).

  python tools/scramjet_long.py --steps 30000 --chunk 2000 [--split] [--dump DIR]

--split runs the split predict / fill pair instead of the lean mechanism step.
A chunk that ends in the Tg < 0 error prints it and stops; with --dump the
fields of the last good chunk (a window around its coldest cell) and of the
failed state are written there as .npz."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ("T", "p", "U", "V", "rho", "mach", "mu_t", "CT")


def coldest(sim, T, n=5):
    """The n coldest active cells, at least 8 cells apart."""
    nx, ny = T.shape
    dx, dy = sim.case.dx, sim.case.dy
    act = np.where(T > 0, T, np.inf)
    order = np.argsort(act, axis=None)[:2000]
    out = []
    for f in order:
        i, j = divmod(int(f), ny)
        if any(abs(i - a) < 8 and abs(j - b) < 8 for a, b, _ in out):
            continue
        out.append((i, j, float(act[i, j])))
        if len(out) == n:
            break
    return ["(%d,%d) x=%.4f y=%.4f T=%.1f" % (i, j, i * dx, j * dy, t) for i, j, t in out]


def window(sim, i0, j0, half=40):
    nx, ny = sim.shape
    a, b = max(0, i0 - half), min(nx, i0 + half)
    out = {"i0": a, "j0": 0}
    for f in FIELDS:
        out[f] = np.asarray(sim.field(f))[a:b, :].astype(np.float32)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--split", action="store_true")
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    if a.split:
        sim.solver.lean_mech = False
    tchem = sim.case.chem_tmin
    done = 0
    last = None
    t0 = time.time()
    while done < a.steps:
        try:
            sim.step(a.chunk)
        except RuntimeError as e:
            print("after %d + <=%d steps: %s" % (done, a.chunk, e), flush=True)
            T = np.asarray(sim.field("T"))
            bad = np.argwhere(~(T > 0))
            print("cells with T <= 0 or nan: %d, first %s" % (len(bad), bad[:5].tolist()), flush=True)
            if a.dump:
                os.makedirs(a.dump, exist_ok=True)
                if last is not None:
                    np.savez_compressed(os.path.join(a.dump, "last_good.npz"), step=last[0], **last[1])
                i0 = int(bad[0][0]) if len(bad) else 0
                np.savez_compressed(os.path.join(a.dump, "failed.npz"), step=done + a.chunk,
                                    **window(sim, i0, 0))
            return 1
        done += a.chunk
        T = np.asarray(sim.field("T"))
        act = T[T > 0]
        print("step %6d dt %.17g  T %.1f .. %.1f  hot %.1f %%  lean steps %d  (%.0f s)" % (
            done, sim.summary()["dt"], act.min(), act.max(), 100 * (T >= tchem).mean(), sim.solver.lnm_steps,
            time.time() - t0), flush=True)
        cold = coldest(sim, T)
        print("   coldest: " + "; ".join(cold), flush=True)
        if a.dump:
            i, j = np.unravel_index(np.argmin(np.where(T > 0, T, np.inf)), T.shape)
            last = (done, window(sim, int(i), int(j)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
