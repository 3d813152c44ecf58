"""Step two backends side by side and report where they diverge.

  python tools/compare_backends.py --a gpu --b cpu --nx 200 --ny 40 --steps 5
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="gpu")
    ap.add_argument("--b", default="cpu")
    ap.add_argument("--nx", type=int, default=200)
    ap.add_argument("--ny", type=int, default=40)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--deck", default=None)
    ap.add_argument("--physics", default="euler")
    ap.add_argument("--no-fused", action="store_true")
    args = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    if args.deck:
        text = open(args.deck, errors="replace").read()
    else:
        ns = args.physics != "euler"
        text = decks.wedge15(args.nx, args.ny, navier_stokes=ns, turbulence=4 if args.physics == "kes" else 0,
                             nmax=10 ** 6, nout=10 ** 5)
    A = hf.Simulation(text, args.a, fused=not args.no_fused)
    B = hf.Simulation(text, args.b)
    for s in range(args.steps):
        A.step(1, residual=True)
        B.step(1, residual=True)
        sa, sb = A.summary(), B.summary()
        line = ["step %d dt %.17g/%.17g" % (s + 1, sa["dt"], sb["dt"])]
        for f in ["rho", "U", "V", "p", "T"]:
            a, b = A.field(f), B.field(f)
            d = np.abs(a - b)
            k = np.unravel_index(np.argmax(d), d.shape)
            line.append("%s %.2e@%s" % (f, d.max() / max(np.abs(b).max(), 1e-300), tuple(int(x) for x in k)))
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
