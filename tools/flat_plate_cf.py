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
ap.add_argument("--cfl", type=float, default=None, help="constant CFL (default: the deck's 0.1 ramp)")
ap.add_argument("--beta0", type=float, default=None, help="DEEPS blending factor beta0 (deck default 0.9875)")
ap.add_argument("--bff", type=int, default=None, help="blending-factor function (deck default 4)")
ap.add_argument("--max-steps", type=int, default=10 ** 9)
ap.add_argument("--sst-d1", type=float, default=None, help="SSTWallDistance (wall omega distance / dy; default 1.0, the Menter first-cell distance)")
ap.add_argument("--wall-blend", type=int, default=0, help="WallBlendCells (near-wall blend of the tangential momentum)")
ap.add_argument("--wall-blend-factor", type=float, default=0.0, help="WallBlendFactor")
ap.add_argument("--out", default="")
a = ap.parse_args()

x_le = 0.2
text = decks.flat_plate(a.nx, a.ny, dx=a.dx, dy=a.dy, x_le=x_le, mach=a.mach, p=a.p, turbulence=a.model,
                        nmax=10 ** 9, nout=10 ** 8, cfl=a.cfl)
# the plate is the domain edge (no solid cells): wall heat transfer has nothing to do, and with
# adiabatic walls the lean N-S kernels apply
text = decks.set_key(text, "isAdiabaticWall", 1)
if a.beta0 is not None:
    text = decks.set_key(text, "beta", a.beta0)
    text = decks.set_table(text, "beta_Scenario", [(0.0, a.beta0), (1.0e9, a.beta0)])
if a.bff is not None:
    text = decks.set_key(text, "BFF", a.bff)
if a.wall_blend:
    text = decks.set_key(text, "WallBlendCells", a.wall_blend)
    text = decks.set_key(text, "WallBlendFactor", a.wall_blend_factor)
if a.sst_d1 is not None:
    text = decks.set_key(text, "SSTWallDistance", a.sst_d1)
sim = hf.Simulation(text, a.backend)
L = a.nx * a.dx
t_end = a.flow_throughs * L / (a.mach * 341.0)
t0 = time.time()
steps = 0
while sim.summary()["time"] < t_end and steps < a.max_steps:
    sim.step(2000)
    steps += 2000
r = validation.plate_cf(sim, x_le)
print("wall blend %d (factor %g)  model %d grid %dx%d dy=%g cfl=%s beta0=%s: %d steps, t=%.3g s (%.1f s wall), lean N-S steps %s" % (
    a.wall_blend, a.wall_blend_factor, a.model, a.nx, a.ny, a.dy, a.cfl, a.beta0, steps, sim.summary()["time"], time.time() - t0,
    getattr(sim.solver, "lns_steps", None)))
print("Mach_e %.2f  Tw/Te %.2f..%.2f" % (r["Mach"][0], r["Tw"].min() / 288.9, r["Tw"].max() / 288.9))
for q in (0.1, 0.25, 0.5, 0.75, 0.9):
    k = int(q * (len(r["x"]) - 1))
    print("Re_x %9.3g  Re_theta %7.0f  Cf/vdII(Re_theta): molecular %.3f  effective %.3f  |  Cf/vdII(Re_x) "
          "molecular %.3f" % (r["Re_x"][k], r["Re_theta"][k], r["Cf"][k] / r["Cf_vd2_theta"][k],
                              r["Cf_eff"][k] / r["Cf_vd2_theta"][k], r["Cf"][k] / r["Cf_turb_vd2"][k]))
    print("Re_x %9.3g  Cf %.4e  Cf/lam %.3f  Cf/turb %.3f  effective (max near-wall stress) Cf/lam %.3f Cf/turb %.3f"
          "  Cf/vdII %.3f" % (
              r["Re_x"][k], r["Cf"][k], r["Cf"][k] / r["Cf_lam"][k], r["Cf"][k] / r["Cf_turb"][k],
              r["Cf_eff"][k] / r["Cf_lam"][k], r["Cf_eff"][k] / r["Cf_turb"][k],
              r["Cf_eff"][k] / r["Cf_turb_vd2"][k]))
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
# near-wall momentum balance at x/L = 0.9: in a zero-pressure-gradient layer the
# total shear stress (mu + mu_t) dU/dy stays ~ tau_w through the viscous and
# buffer layers; a rise above tau_w away from the wall means the scheme's own
# (numerical) diffusion carries part of the wall stress
U = np.asarray(sim.field("U"))
mu_, rho_ = np.asarray(sim.field("mu")), np.asarray(sim.field("rho"))
mut_ = np.asarray(sim.field("mu_t")) if a.model else np.zeros_like(mu_)
i = int(0.2 * U.shape[0] + 0.9 * 0.8 * U.shape[0])
tw = mu_[i, 0] * (U[i, 1] - U[i, 0]) / a.dy
ut = np.sqrt(abs(tw) / rho_[i, 0])
# the DEEPS blend's own diffusion across the first cell: (1 - beta) dyy/2 dy^2/dt (beta ~ beta0)
beta0 = float(a.beta0) if a.beta0 is not None else 0.9875
dyy = a.dx / (a.dx + a.dy)
d_num = (1.0 - beta0) * dyy * 0.5 * a.dy ** 2 / sim.summary()["dt"]
nu_w = mu_[i, 0] / rho_[i, 0]
print("x/L 0.92: tau_w %.4g Pa, u_tau %.3g m/s, blend diffusion / nu_w at the wall %.2f" % (tw, ut, d_num / nu_w))
print("  j, y+, U+, (mu+mu_t) dU/dy / tau_w:")
for j in (1, 2, 3, 5, 8, 12, 20, 30, 45, 70):
    if j + 1 >= U.shape[1]:
        break
    tt = (mu_[i, j] + mut_[i, j]) * (U[i, j + 1] - U[i, j - 1]) / (2 * a.dy)
    print("  j %3d  y+ %7.2f  U+ %6.2f  tau/tau_w %.3f" % (j, j * a.dy * ut * rho_[i, 0] / mu_[i, 0], U[i, j] / ut,
                                                        tt / tw))
if a.out:
    with open(a.out, "w") as f:
        json.dump({k: np.asarray(v).tolist() for k, v in r.items()} | {"model": a.model, "steps": steps}, f)
