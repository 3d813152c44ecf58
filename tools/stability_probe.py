"""Step a generated deck on the GPU and report when/where it goes unstable.
  python tools/stability_probe.py scramjet 6000 400 --steps 400 --set TurbulenceModel=4"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("deck")
    ap.add_argument("nx", type=int)
    ap.add_argument("ny", type=int)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--chunk", type=int, default=50)
    ap.add_argument("--backend", default="gpu")
    ap.add_argument("--kw", action="append", default=[], help="generator kwarg k=v (int)")
    ap.add_argument("--set", action="append", default=[], help="deck key k=v")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    kw = {k: int(v) for k, v in (x.split("=") for x in a.kw)}
    text = decks.GENERATORS[a.deck](a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8, **kw)
    for x in a.set:
        k, v = x.split("=")
        text = decks.set_key(text, k, float(v) if "." in v or "e" in v else int(v))
    s = hf.Simulation(text, a.backend)
    done = 0
    while done < a.steps:
        try:
            s.step(a.chunk, residual=True)
        except Exception as e:
            print("UNSTABLE after <= %d steps: %s" % (done + a.chunk, e), flush=True)
            T = s.field("T")
            sol = s.field("solid") > 0
            bad = np.argwhere((~sol) & ((T < 0) | ~np.isfinite(T)))
            print("bad cells:", bad[:10].tolist(), flush=True)
            return 1
        done += a.chunk
        T = s.field("T")
        sol = s.field("solid") > 0
        j = np.unravel_index(np.argmax(np.where(sol, -1, T)), T.shape)
        print("step %d  Tmax %.1f at %s  max_rms %.3g  dt %.3g" % (done, T[j], tuple(int(x) for x in j),
                                                                  s.summary()["max_rms"], s.summary()["dt"]),
              flush=True)
    print("STABLE %d steps" % done)
    return 0


if __name__ == "__main__":
    sys.exit(main())
