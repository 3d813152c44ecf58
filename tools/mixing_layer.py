"""Compressible mixing-layer spreading rate on the GPU (models/validation.py
mixing_layer_growth): runs decks.mixing_layer for a number of slow-stream
flow-through times and prints the vorticity-thickness growth rate against
the incompressible and the convective-Mach-corrected correlations."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks, validation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", type=int, default=6, help="TurbulenceModel code: 0 laminar, 4 k-eps, 6 SST")
ap.add_argument("--nx", type=int, default=600)
ap.add_argument("--ny", type=int, default=300)
ap.add_argument("--dx", type=float, default=5e-4)
ap.add_argument("--dy", type=float, default=1e-4)
ap.add_argument("--m1", type=float, default=2.0)
ap.add_argument("--m2", type=float, default=1.2)
ap.add_argument("--p", type=float, default=5e4)
ap.add_argument("--flow-throughs", type=float, default=2.5)
ap.add_argument("--backend", default="gpu")
ap.add_argument("--out", default="")
ap.add_argument("--no-lean-ns", action="store_true")
a = ap.parse_args()

text = decks.mixing_layer(a.nx, a.ny, dx=a.dx, dy=a.dy, mach1=a.m1, mach2=a.m2, p=a.p, turbulence=a.model,
                          nmax=10 ** 9, nout=10 ** 8)
sim = hf.Simulation(text, a.backend)
if a.no_lean_ns:
    sim.solver.lean_ns = False
L = a.nx * a.dx
t_end = a.flow_throughs * L / (a.m2 * 347.0)
t0 = time.time()
steps = 0
while sim.summary()["time"] < t_end:
    sim.step(2000)
    steps += 2000
    if steps % 20000 == 0:
        g = validation.mixing_layer_growth(sim)
        print("  %d steps t=%.3g s: rate %.4f r2 %.3f" % (steps, sim.summary()["time"], g["rate"], g["r2"]), flush=True)
g = validation.mixing_layer_growth(sim)
print("model %d grid %dx%d: %d steps, t=%.3g s (%.1f s wall)" % (a.model, a.nx, a.ny, steps, sim.summary()["time"],
                                                               time.time() - t0))
print("U1 %.1f U2 %.1f lambda %.3f Mc %.3f" % (g["U1"], g["U2"], g["lambda"], g["Mc"]))
print("d(delta_w)/dx = %.4f (R^2 %.3f); incompressible 0.18*lambda = %.4f (ratio %.2f); "
      "Langley-corrected %.4f (ratio %.2f)" % (g["rate"], g["r2"], g["rate_incompressible"],
                                               g["rate"] / g["rate_incompressible"], g["rate_compressible"],
                                               g["rate"] / g["rate_compressible"]))
mut, mu = np.asarray(sim.field("mu_t")), np.asarray(sim.field("mu"))
for q in (0.3, 0.6, 0.9):
    i = int(q * a.nx)
    print("x/L %.1f delta_w %.3e m  max mu_t/mu %.1f" % (q, g["delta_w"][min(len(g["x"]) - 1, max(0, i - int(0.3 * a.nx)))],
                                                       (mut[i] / mu[i]).max()))
if a.out:
    with open(a.out, "w") as f:
        json.dump({k: (np.asarray(v).tolist() if isinstance(v, np.ndarray) else v) for k, v in g.items()}
                  | {"model": a.model, "steps": steps}, f)
