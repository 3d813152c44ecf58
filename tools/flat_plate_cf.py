"""Flat-plate skin friction on the GPU against laminar / turbulent correlations
(models/validation.py).  Prints Cf / Cf_correlation at Re_x stations and
writes the profiles as JSON (--out)."""
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
ap.add_argument("--model", type=int, default=0, help="TurbulenceModel code: 0 laminar, 4 k-eps, 6 SST")
ap.add_argument("--nx", type=int, default=250)
ap.add_argument("--ny", type=int, default=100)
ap.add_argument("--dx", type=float, default=1e-3)
ap.add_argument("--dy", type=float, default=1e-4)
ap.add_argument("--p", type=float, default=1e3)
ap.add_argument("--mach", type=float, default=2.5)
ap.add_argument("--flow-throughs", type=float, default=3.0)
ap.add_argument("--backend", default="gpu")
ap.add_argument("--out", default="")
a = ap.parse_args()

x_le = 0.2
text = decks.flat_plate(a.nx, a.ny, dx=a.dx, dy=a.dy, x_le=x_le, mach=a.mach, p=a.p, turbulence=a.model,
                        nmax=10 ** 9, nout=10 ** 8)
sim = hf.Simulation(text, a.backend)
L = a.nx * a.dx
t_end = a.flow_throughs * L / (a.mach * 341.0)
t0 = time.time()
steps = 0
while sim.summary()["time"] < t_end:
    sim.step(2000)
    steps += 2000
r = validation.plate_cf(sim, x_le)
print("model %d grid %dx%d dy=%g: %d steps, t=%.3g s (%.1f s wall)" % (a.model, a.nx, a.ny, a.dy, steps,
                                                                     sim.summary()["time"], time.time() - t0))
print("Mach_e %.2f  Tw/Te %.2f..%.2f" % (r["Mach"][0], r["Tw"].min() / 288.9, r["Tw"].max() / 288.9))
for q in (0.1, 0.25, 0.5, 0.75, 0.9):
    k = int(q * (len(r["x"]) - 1))
    print("Re_x %9.3g  Cf %.4e  Cf/lam %.3f  Cf/turb %.3f" % (r["Re_x"][k], r["Cf"][k], r["Cf"][k] / r["Cf_lam"][k],
                                                              r["Cf"][k] / r["Cf_turb"][k]))
if a.model:
    mut, mu, yp = (np.asarray(sim.field(f)) for f in ("mu_t", "mu", "y_plus"))
    k_ = np.asarray(sim.field("S7")) / np.asarray(sim.field("rho"))
    nx = mut.shape[0]
    for q in (0.25, 0.5, 0.9):
        i = int(0.2 * nx + q * 0.8 * nx)
        r_ = mut[i] / mu[i]
        print("x/L %.2f  max mu_t/mu %.1f at j=%d  y+(1)=%.2f  k max %.3g at j=%d  U(j=1..5)=%s" % (
            i / nx, r_.max(), int(r_.argmax()), yp[i, 1], k_[i].max(), int(k_[i].argmax()),
            np.array2string(np.asarray(sim.field("U"))[i, 1:6], precision=1)))
if a.out:
    with open(a.out, "w") as f:
        json.dump({k: np.asarray(v).tolist() for k, v in r.items()} | {"model": a.model, "steps": steps}, f)
