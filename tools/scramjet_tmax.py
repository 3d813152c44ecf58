"""Where and why the SCRAMJET deck's maximum temperature sits where it does.

Runs the 6000x400 scramjet deck on the GPU in the reference's 4-slot model
(one-step global H2/air reaction, no dissociation) and in mechanism mode
(9 species / 21 reversible steps, thermally perfect NASA-7 gas) and prints,
every --every steps, Tmax, its cell, the local Mach number and (mechanism
mode) the local H2O / OH / H2 mass fractions, next to the inflow stagnation
temperature T0 = T (1 + (k-1)/2 M^2) of the Mach-8 air stream."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=3000)
ap.add_argument("--every", type=int, default=300)
ap.add_argument("--nx", type=int, default=6000)
ap.add_argument("--ny", type=int, default=400)
a = ap.parse_args()

T_inf, M_inf = 226.5, 8.0
for k in (1.4, 1.33):
    print("inflow stagnation temperature (k=%.2f): %.0f K" % (k, T_inf * (1 + 0.5 * (k - 1) * M_inf ** 2)))
for mode in ("4-slot", "mechanism"):
    text = decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8, mechanism=None if mode == "4-slot" else "h2_air_li2004")
    sim = hf.Simulation(text, "gpu")
    print("== %s ==" % mode, flush=True)
    done = 0
    while done < a.steps:
        sim.step(a.every)
        done += a.every
        T = sim.field("T")
        i, j = np.unravel_index(np.argmax(T), T.shape)
        mach = sim.field("mach")[i, j]
        extra = ""
        if mode == "mechanism":
            ys = {s: sim.field("Y:" + s)[i, j] for s in ("H2O", "OH", "H2", "O2")}
            extra = "  Y(H2O,OH,H2,O2)=(%.3f, %.4f, %.4f, %.3f)" % tuple(ys.values())
        else:
            extra = "  Y_cp=%.3f" % (sim.field("S6")[i, j] / max(sim.field("rho")[i, j], 1e-300))
        s = sim.summary()
        print("step %5d  Tmax %7.1f K at (%d, %d)  Mach %.2f  dt %.3g%s" % (done, T[i, j], i, j, mach, s["dt"], extra),
              flush=True)
