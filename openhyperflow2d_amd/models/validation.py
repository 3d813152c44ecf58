"""Flat-plate skin friction against boundary-layer correlations (validation of
the viscous discretisation and of the turbulence models).

The plate deck is ``decks.flat_plate``: no-slip wall along y = 0 from the
leading edge ``x_le`` to the outlet, uniform supersonic free stream.  The wall
shear is taken from the first cell above the wall, tau_w = mu_w (U_1 - U_0)/dy
(U_0 = 0 on the no-slip node), and Cf = tau_w / (rho_e U_e^2 / 2) with the
free-stream state read at the inflow.

Correlations, with Eckert's reference temperature for compressibility
(T*/T_e = 0.5 + 0.039 M_e^2 + 0.5 T_w/T_e, Sutherland viscosity):
  laminar (Blasius)       Cf = 0.664 sqrt(C*) / sqrt(Re_x),  C* = rho* mu* / (rho_e mu_e)
  turbulent (Schlichting) Cf = 0.0592 (rho*/rho_e) (Re_x*)^-0.2,  Re_x* = rho* U_e x / mu*
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np


def sutherland(T: float) -> float:
    return 1.716e-5 * (T / 273.15) ** 1.5 * (273.15 + 110.4) / (T + 110.4)


def plate_cf(sim, x_le_frac: float) -> Dict[str, np.ndarray]:
    """Cf, Re_x and the correlations along the plate of a flat_plate run."""
    case = sim.case
    dx, dy = case.dx, case.dy
    U, rho, mu, T = (np.asarray(sim.field(f)) for f in ("U", "rho", "mu", "T"))
    p = np.asarray(sim.field("p"))
    nx, ny = U.shape
    i_le = int(round(x_le_frac * nx))
    # free stream: inflow column, mid height
    je = ny // 2
    Ue, rhoe, mue, Te, pe = U[0, je], rho[0, je], mu[0, je], T[0, je], p[0, je]
    ae = math.sqrt(1.4 * pe / rhoe)
    Me = Ue / ae
    i = np.arange(i_le + 1, nx - 2)
    x = (i - i_le) * dx
    tau = mu[i, 0] * (U[i, 1] - U[i, 0]) / dy
    cf = tau / (0.5 * rhoe * Ue * Ue)
    rex = rhoe * Ue * x / mue
    Tw = T[i, 0]
    Ts = Te * (0.5 + 0.039 * Me * Me + 0.5 * Tw / Te)
    mus = np.array([sutherland(t) for t in Ts])
    rhos = rhoe * Te / Ts
    cstar = rhos * mus / (rhoe * mue)
    lam = 0.664 * np.sqrt(cstar) / np.sqrt(rex)
    turb = 0.0592 * (rhos / rhoe) * (rhos * Ue * x / mus) ** -0.2
    return {"x": x, "Re_x": rex, "Cf": cf, "Cf_lam": lam, "Cf_turb": turb, "Mach": np.full_like(x, Me),
            "Tw": Tw}
