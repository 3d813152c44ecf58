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
and, as a second compressible turbulent reference, van Driest II (van_driest_ii).
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np


def sutherland(T: float) -> float:
    return 1.716e-5 * (T / 273.15) ** 1.5 * (273.15 + 110.4) / (T + 110.4)


def van_driest_ii(re_x, mach: float, Te: float, Tw, r: float = 0.89, gamma: float = 1.4):
    """Turbulent flat-plate Cf by the van Driest II transformation (Hopkins &
    Inouye's form): Cf = Cf_inc(F_Rx Re_x) / F_c with
      m = (gamma-1)/2 M^2,  T_aw/T_e = 1 + r m,
      A = (r m T_e/T_w)^1/2,  B = T_aw/T_w - 1,
      alpha = (2A^2 - B)/(4A^2 + B^2)^1/2,  beta = B/(4A^2 + B^2)^1/2,
      F_c = (T_aw/T_e - 1) / (asin alpha + asin beta)^2,
      F_Rx = (mu_e/mu_w) / F_c  (Sutherland viscosities),
    and the same incompressible law as the Eckert comparison, Cf_inc = 0.0592 Re^-0.2."""
    re_x = np.asarray(re_x, dtype=np.float64)
    Tw = np.asarray(Tw, dtype=np.float64)
    m = 0.5 * (gamma - 1.0) * mach * mach
    taw_te = 1.0 + r * m
    a = np.sqrt(r * m * Te / Tw)
    b = taw_te * Te / Tw - 1.0
    den = np.sqrt(4.0 * a * a + b * b)
    fc = (taw_te - 1.0) / (np.arcsin((2.0 * a * a - b) / den) + np.arcsin(b / den)) ** 2
    mu_w = np.array([sutherland(t) for t in np.atleast_1d(Tw)]).reshape(Tw.shape)
    frx = (sutherland(Te) / mu_w) / fc
    return 0.0592 * (frx * re_x) ** -0.2 / fc


def _vd2_factors(mach: float, Te: float, Tw, r: float = 0.89, gamma: float = 1.4):
    """(F_c, F_theta = mu_e / mu_w) of the van Driest II transformation."""
    Tw = np.asarray(Tw, dtype=np.float64)
    m = 0.5 * (gamma - 1.0) * mach * mach
    taw_te = 1.0 + r * m
    a = np.sqrt(r * m * Te / Tw)
    b = taw_te * Te / Tw - 1.0
    den = np.sqrt(4.0 * a * a + b * b)
    fc = (taw_te - 1.0) / (np.arcsin((2.0 * a * a - b) / den) + np.arcsin(b / den)) ** 2
    mu_w = np.array([sutherland(t) for t in np.atleast_1d(Tw)]).reshape(Tw.shape)
    return fc, sutherland(Te) / mu_w


def van_driest_ii_theta(re_theta, mach: float, Te: float, Tw, r: float = 0.89, gamma: float = 1.4):
    """Turbulent Cf against the momentum-thickness Reynolds number: van Driest
    II with the Karman-Schoenherr law, Cf = Cf_KS(F_theta Re_theta) / F_c,
    1 / Cf_KS = 17.08 (log10 Re)^2 + 25.11 log10 Re + 6.012.  Unlike the Re_x
    forms it does not assume a layer turbulent from the leading edge: the
    local state of the layer (theta) carries its history, so a delayed
    transition (the virtual origin of the turbulent layer) drops out."""
    fc, ft = _vd2_factors(mach, Te, Tw, r, gamma)
    lg = np.log10(ft * np.asarray(re_theta, dtype=np.float64))
    return 1.0 / (17.08 * lg * lg + 25.11 * lg + 6.012) / fc


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
    # Diagnostic only (the validation asserts on the molecular Cf above): the
    # modelled stress (mu + mu_t) dU/dy averaged over 30 <= y+ <= 100.  The
    # DEEPS predictor blends every conserved variable with its neighbours'
    # mean by (1 - beta), a diffusion (1 - beta) dyy / 2 * dy^2 / dt
    # (dyy = dx / (dx + dy)) in parallel with the molecular one: in the
    # viscous sublayer it carries part of the wall stress, so mu_w dU/dy sees
    # only the rest, while in a zero-pressure-gradient layer the total stress
    # stays ~ tau_w through the log layer (profiles/flat_plate_validation.md).
    mut = np.asarray(sim.field("mu_t"))
    uplus_tau = np.sqrt(np.abs(tau) / rho[i, 0])
    tau_eff = np.abs(tau).copy()
    for q, ii in enumerate(i):
        yplus = np.arange(ny) * dy * uplus_tau[q] * rho[ii, 0] / mu[ii, 0]
        band = [j for j in range(1, ny - 1) if 30.0 <= yplus[j] <= 100.0]
        if band:
            tau_eff[q] = float(np.mean([(mu[ii, j] + mut[ii, j]) * (U[ii, j + 1] - U[ii, j - 1]) / (2 * dy)
                                        for j in band]))
    cf_eff = np.sign(cf) * tau_eff / (0.5 * rhoe * Ue * Ue)
    # momentum thickness theta = int rho U / (rho_e U_e) (1 - U / U_e) dy over
    # the layer (up to the first node at 0.995 U_e, the inflow edge state)
    theta = np.zeros(len(i))
    for q, ii in enumerate(i):
        ru = rho[ii] * U[ii] / (rhoe * Ue) * (1.0 - U[ii] / Ue)
        top = np.nonzero(U[ii, 1:] >= 0.995 * Ue)[0]
        jt = int(top[0]) + 1 if len(top) else ny - 1
        theta[q] = float(np.sum(ru[:jt + 1]) * dy)
    re_theta = rhoe * Ue * theta / mue
    # the DEEPS blend's own diffusion across the first cell off the wall,
    # (1 - beta) dyy/2 dy^2/dt with the rho U blending factor there, against
    # the molecular nu_w: the near-wall error driver of the molecular Cf
    beta1 = np.asarray(sim.field("beta1"))
    dyy = dx / (dx + dy)
    d_num = (1.0 - beta1[i, 1]) * dyy * 0.5 * dy * dy / sim.summary()["dt"]
    blend_nu = d_num / (mu[i, 0] / rho[i, 0])
    return {"x": x, "Re_x": rex, "Cf": cf, "Cf_eff": cf_eff, "Cf_lam": lam, "Cf_turb": turb, "blend_nu": blend_nu,
            "Cf_turb_vd2": van_driest_ii(rex, Me, Te, Tw), "theta": theta, "Re_theta": re_theta,
            "Cf_vd2_theta": van_driest_ii_theta(re_theta, Me, Te, Tw), "Mach": np.full_like(x, Me), "Tw": Tw}


def extrapolate_to_zero(xs, ys):
    """Value at x = 0 of the polynomial (degree len - 1, at most 2) through
    the points (x, y): the zero-blend-diffusion limit of a grid sequence."""
    xs = np.asarray(xs, dtype=np.float64)
    ys = np.asarray(ys, dtype=np.float64)
    return float(np.polyval(np.polyfit(xs, ys, min(len(xs) - 1, 2)), 0.0))


def langley_phi(mc: float) -> float:
    """Compressibility reduction of the mixing-layer growth rate, the usual
    fit to the Langley experimental curve: 0.23 + 0.77 exp(-3.5 Mc^2)."""
    return 0.23 + 0.77 * math.exp(-3.5 * mc * mc)


def mixing_layer_growth(sim, x0_frac: float = 0.3, x1_frac: float = 0.9) -> Dict[str, object]:
    """Vorticity thickness delta_w(x) = (U1 - U2) / max_y |dU/dy| of a
    ``decks.mixing_layer`` run, its linear growth rate over [x0, x1] of the
    domain and the reference rates: incompressible
    d(delta_w)/dx = 0.18 lambda (lambda = (U1 - U2)/(U1 + U2), equal
    densities; Brown & Roshko) and the compressible one scaled by the
    convective-Mach fit langley_phi(Mc), Mc = (U1 - U2)/(a1 + a2)."""
    case = sim.case
    dx, dy = case.dx, case.dy
    U, rho, p = (np.asarray(sim.field(f)) for f in ("U", "rho", "p"))
    nx, ny = U.shape
    U1, U2 = U[0, ny - 3], U[0, 2]
    a1 = math.sqrt(1.4 * p[0, ny - 3] / rho[0, ny - 3])
    a2 = math.sqrt(1.4 * p[0, 2] / rho[0, 2])
    dU = U1 - U2
    i = np.arange(int(x0_frac * nx), int(x1_frac * nx))
    grad = np.abs(np.diff(U[i, 2:ny - 2], axis=1)) / dy
    dw = dU / grad.max(axis=1)
    x = (i + 0.5) * dx
    A = np.vstack([x, np.ones_like(x)]).T
    coef, res, _, _ = np.linalg.lstsq(A, dw, rcond=None)
    pred = A @ coef
    r2 = 1.0 - float(((dw - pred) ** 2).sum()) / float(((dw - dw.mean()) ** 2).sum() + 1e-300)
    lam = dU / (U1 + U2)
    mc = dU / (a1 + a2)
    inc = 0.18 * lam
    return {"x": x, "delta_w": dw, "rate": float(coef[0]), "r2": r2, "lambda": lam, "Mc": mc,
            "rate_incompressible": inc, "rate_compressible": inc * langley_phi(mc), "U1": U1, "U2": U2}
