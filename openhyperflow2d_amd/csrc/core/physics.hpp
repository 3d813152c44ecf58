// Pointwise cell physics shared by the host (CPU oracle / pre-processor) and
// the HIP kernels: primitive recovery, wall treatment, inviscid + viscous flux
// assembly, the RANS/LES turbulence closures and the Zeldovich chemistry with
// mixture-property update.
//
// Behavioural reference (re-derived, not translated):
//   FillNode2D            libOpenHyperFLOW2D/hyper_flow_node.hpp:373-600
//   TurbModRANS2D         libOpenHyperFLOW2D/hyper_flow_node.hpp:601-957
//   TurbulenceAxisymmAddOn hyper_flow_node.hpp:241-252
//   CalcChemicalReactions libDEEPS2D/deeps2d_core.cpp:4697-4780
//
// Every function is templated on the node type N; both the 1248-byte host
// CellRecord and the register-resident device CellLocal expose the same member
// names, so a single source of truth drives CPU and GPU numerics.
#pragma once

#include <cmath>
#include "common.hpp"

namespace hf2d {

struct FillParams {
  int is_mu_t = 0;
  int is_init = 0;
  real sig_w = 0.0;
  real sig_f = 0.0;
  int tem = TEM_k_eps_Std;
  real delta = 0.0;
  int sm = SM_NS;
  int FT = FT_FLAT;       // static FlowNode2D::FT
  real dx = 1.0, dy = 1.0;
  real Hu[NSPEC] = {0, 0, 0, 0};
  int isSrcAdd = 0;
  real turb_I = 0.005;    // FlowNodeTurbulence2D::I
  int sst_version = 2003; // new model (not in reference)
  real sst_d1 = 1.0;      // SST wall omega distance / min(dx, dy) (Config::SSTWallDistance)
  real dt = 0.0;          // time step of the fill's step (SST point-implicit destruction)
};

HF_HD inline real hf_max(real a, real b) { return a > b ? a : b; }

// x^n for an integer exponent the way the reference's C++98 build evaluates
// pow(double, int) (libgcc __powidf2: binary powering, e.g. x^6 = x^2 * x^4),
// which differs from libm pow in the last bits.
HF_HD inline real powi_ref(real x, int m) {
  unsigned n = m < 0 ? 0u - (unsigned)m : (unsigned)m;
  real y = (n % 2) ? x : 1.0;
  while (n >>= 1) {
    x = x * x;
    if (n % 2) y = y * x;
  }
  return m < 0 ? 1.0 / y : y;
}
HF_HD inline real hf_min(real a, real b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------
// Axisymmetric turbulence add-on (diffusive F terms for k/eps or nu~).
// ---------------------------------------------------------------------------
template <class N>
HF_HD inline void turb_axisym_addon(N& n, const FillParams& P, int is_init) {
  const real FT = (real)P.FT;
  if (has_all(n.TurbType, TCT_k_eps_Model) && !is_init) {
    n.F[I_K] = FT * (n.mu + n.mu_t) * n.dkdy;
    n.F[I_EPS] = FT * (n.mu + hf_div(n.mu_t, 1.3)) * n.depsdy;
  } else if (has_all(n.TurbType, TCT_Spalart_Allmaras_Model) && !is_init) {
    n.F[I_NUT] = FT * (n.mu / n.S[I_RHO] + n.S[I_NUT]) * n.dkdy;
  } else if (is_init) {
    n.F[I_NUT] = n.F[I_EPS] = 0.0;
    n.Src[I_NUT] = n.Src[I_EPS] = 0.0;
  }
}

// Menter k-omega SST (new physics, no reference counterpart: the reference
// reserves TCT_k_omega_SST_Model_2D / TEM_k_omega_SST but leaves the branch
// empty, hyper_flow_node.hpp:919-926).  omega lives in the eps slot (i2d_omega
// alias, hyper_flow_turbulence.hpp:20).  Conserved variables are rho*k and
// rho*omega; the blending functions use the wall distance l_min.
template <class N>
HF_HD inline void turb_sst(N& n, const FillParams& P, int is_mu_t, int is_init) {
  const real sk1 = 0.85, so1 = 0.5, b1 = 0.075;
  const real sk2 = 1.0, so2 = 0.856, b2 = 0.0828;
  const real bstar = 0.09, a1 = 0.31, kappa = 0.41;
  const real rho = n.S[I_RHO];
  const real dmin = hf_max(n.l_min, 1e-12);
  // Free-stream / inflow omega: the mixing-length estimate, but never below
  // k / (10 nu) (eddy-viscosity ratio <= 10, Menter's free-stream range).  A
  // larger ratio at a Mach-8, low-density inflow (nu ~ 1e-3 m^2/s) makes the
  // explicit viscous number nu_t dt / dx^2 exceed the stability bound on
  // 0.1 mm grids, since dt follows the inviscid CFL only.
  auto omega_inflow = [&](real kk_, real l_) {
    return hf_max(std::sqrt(kk_) / (std::pow(bstar, 0.25) * l_), hf_max(kk_ / (10.0 * n.mu / rho + 1e-300), 1e-6));
  };
  if (is_init) {
    const real TmpI = P.turb_I * std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
    const real kk = 1.5 * TmpI * TmpI;
    const real l = hf_max(n.l_min, hf_min(P.dx, P.dy)) * 0.41;
    const real om = omega_inflow(kk, l);
    n.S[I_K] = rho * kk;
    n.S[I_OMEGA] = rho * om;
    n.mu_t = (om > 0) ? rho * kk / om : 0.0;
    return;
  }
  if (has_all(n.CT, CT_WALL_NO_SLIP) || has_all(n.CT, CT_WALL_LAW)) {
    // Menter wall BC: k = 0, omega = 60 nu / (beta1 d^2)
    const real d1 = hf_min(P.dx, P.dy) * P.sst_d1;
    n.S[I_K] = 0.0;
    n.S[I_OMEGA] = rho * 60.0 * (n.mu / rho) / (b1 * d1 * d1);
  }
  if (has_all(n.TurbType, TCT_k_CONST)) {
    const real TmpI = P.turb_I * std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
    n.S[I_K] = 1.5 * TmpI * TmpI * rho;
  }
  const real kk = hf_max(hf_div(n.S[I_K], rho), 0.0);
  const real nu = hf_div(n.mu, rho);
  // omega floor: eddy-viscosity ratio nu_t / nu <= 1e5 (keeps the explicit
  // cross-diffusion and production terms bounded where k ~ 0, e.g. fluid at
  // rest next to an impulsively started free stream)
  const real om_floor = hf_max(hf_div(kk, 1.0e5 * nu + 1e-300), 1e-6);
  const real om = hf_max(hf_div(n.S[I_OMEGA], rho), om_floor);
  if (has_all(n.TurbType, TCT_eps_CONST)) {
    const real l = hf_max(n.l_min, hf_min(P.dx, P.dy)) * 0.41;
    n.S[I_OMEGA] = rho * hf_max(omega_inflow(kk, l), om_floor);
  }
  // dkdx.. hold d(k)/dx and d(omega)/dx (already divided by rho, like the k-eps path)
  const real cross = n.dkdx * n.depsdx + n.dkdy * n.depsdy;
  const real CDkw = hf_max(hf_div(2.0 * rho * so2, om) * cross, 1e-10);
  const real arg1a = hf_div(hf_sqrt(kk), bstar * om * dmin);
  const real arg1b = hf_div(500.0 * nu, dmin * dmin * om);
  const real arg1 = hf_min(hf_max(arg1a, arg1b), hf_div(4.0 * rho * so2 * kk, CDkw * dmin * dmin));
  const real F1 = std::tanh(arg1 * arg1 * arg1 * arg1);
  const real arg2 = hf_max(2.0 * arg1a, arg1b);
  const real F2 = std::tanh(arg2 * arg2);
  const real Sxy = 0.5 * (n.dUdy + n.dVdx);
  real Smag2 = 2.0 * (n.dUdx * n.dUdx + n.dVdy * n.dVdy) + 4.0 * Sxy * Sxy;
  if (P.FT) Smag2 += 2.0 * hf_div(n.V, n.y) * hf_div(n.V, n.y);
  const real Smag = hf_sqrt(Smag2);
  const real mut = hf_div(rho * a1 * kk, hf_max(a1 * om, Smag * F2));
  const real sk = F1 * sk1 + (1.0 - F1) * sk2;
  const real so = F1 * so1 + (1.0 - F1) * so2;
  const real beta = F1 * b1 + (1.0 - F1) * b2;
  const real gam1 = b1 / bstar - so1 * kappa * kappa / std::sqrt(bstar);
  const real gam2 = b2 / bstar - so2 * kappa * kappa / std::sqrt(bstar);
  const real gam = F1 * gam1 + (1.0 - F1) * gam2;
  real Pk = mut * Smag2;
  Pk = hf_min(Pk, 10.0 * bstar * rho * kk * om);
  if (is_mu_t) {
    n.mu_t = hf_max(0.0, mut);
    n.lam_t = n.mu_t * n.CP;
  }
  n.A[I_K] = n.S[I_K] * n.U;
  n.A[I_OMEGA] = n.S[I_OMEGA] * n.U;
  n.B[I_K] = n.S[I_K] * n.V;
  n.B[I_OMEGA] = n.S[I_OMEGA] * n.V;
  n.RX[I_K] = (n.mu + mut * sk) * n.dkdx;
  n.RX[I_OMEGA] = (n.mu + mut * so) * n.depsdx;
  n.RY[I_K] = (n.mu + mut * sk) * n.dkdy;
  n.RY[I_OMEGA] = (n.mu + mut * so) * n.depsdy;
  n.A[I_K] -= n.RX[I_K];
  n.A[I_OMEGA] -= n.RX[I_OMEGA];
  n.B[I_K] -= n.RY[I_K];
  n.B[I_OMEGA] -= n.RY[I_OMEGA];
  n.SrcAdd[I_K] = n.SrcAdd[I_OMEGA] = 0.0;
  // Point-implicit (Patankar) destruction: with the explicit DEEPS update the
  // sink rho*phi*r (r = beta* omega for k, beta omega for omega) is applied as
  // rho*phi*r / (1 + dt r), i.e. phi_new = phi / (1 + dt r) for the sink alone,
  // which can never drive k or omega negative however large omega gets next to
  // a no-slip wall (omega_w = 60 nu / (beta1 d^2)) on fine grids.
  const real rk = bstar * om, rw = beta * om;
  const real ik = P.dt > 0 ? hf_div(1.0, 1.0 + P.dt * rk) : 1.0;
  const real iw = P.dt > 0 ? hf_div(1.0, 1.0 + P.dt * rw) : 1.0;
  if (!has_all(n.TurbType, TCT_k_CONST)) n.Src[I_K] = Pk - rho * kk * rk * ik;
  if (!has_all(n.TurbType, TCT_eps_CONST)) {
    // production gamma * rho * S^2 (the Pk limiter applied through nu_t) and
    // the cross-diffusion term, each bounded by the destruction scale
    // beta* rho omega^2 * 10 for the explicit DEEPS update
    const real cap = 10.0 * bstar * rho * om * om;
    const real Pw = hf_min(hf_div(gam * rho, hf_max(mut, 1e-30)) * Pk, cap);
    const real CD = hf_max(hf_min(hf_div(2.0 * (1.0 - F1) * rho * so2, om) * cross, cap), -cap);
    n.Src[I_OMEGA] = Pw - rho * om * rw * iw + CD;
  }
  const real FT = (real)P.FT;
  n.F[I_K] = FT * (n.mu + mut * sk) * n.dkdy;
  n.F[I_OMEGA] = FT * (n.mu + mut * so) * n.depsdy;
}

// Spalart-Allmaras branch of TurbModRANS2D (hyper_flow_node.hpp:822-918):
// nu~ in the k slot.
template <class N>
HF_HD inline void turb_sa(N& n, const FillParams& P, int is_mu_t, int is_init) {
  const u64 TT = n.TurbType;
  real fv1 = 1.0;
  if (is_init) {
    n.S[I_NUT] = n.mu / n.S[I_RHO] / 100.0;
  } else if (has_all(n.CT, CT_WALL_NO_SLIP) || has_all(n.CT, CT_WALL_LAW) ||
             has_all(TT, TCT_nu_t_CONST)) {
    n.S[I_NUT] = 0.;
  } else if (has_all(n.CT, NT_FC)) {
    n.S[I_NUT] = n.mu / n.S[I_RHO] * P.turb_I;
  } else {
    const real Cb1 = 0.1355, Cb2 = 0.622, sig = 2.0 / 3.0, _k = 0.41;
    const real Cw1 = Cb1 / (_k * _k) + (1 + Cb2) / sig;
    const real Cw2 = 0.3, Cw3 = 2.0, Cv1 = 7.1, Ct2 = 2.0, Ct4 = 0.5, C5 = 3.5;
    const real a_sound2 = n.k * n.R * n.Tg;
    const real nu = n.mu / n.S[I_RHO];
    const real ksi = n.S[I_NUT] / nu;
    fv1 = ksi * ksi * ksi / (ksi * ksi * ksi + Cv1 * Cv1 * Cv1);
    const real nu_hat = n.mu_t / n.S[I_RHO] / fv1;
    const real fv2 = 1.0 - ksi / (1.0 + ksi * fv1);
    const real Wxy = 0.5 * (n.dVdx - n.dUdy);
    const real Omega = std::sqrt(2.0 * Wxy * Wxy);
    real S_hat = Omega + n.S[I_NUT] / (_k * _k * n.l_min * n.l_min) * fv2;
    if (S_hat < 0.3 * Omega) S_hat = 0.3 * Omega;
    const real r = hf_min((n.S[I_NUT] / (S_hat * _k * _k * n.l_min * n.l_min)), 10.0);
    const real g = r + Cw2 * (std::pow(r, 6.0) - r);
    const real fw = g * std::pow((1.0 + std::pow(Cw3, 6.0)) / (std::pow(g, 6.0) + std::pow(Cw3, 6.0)),
                                 1.0 / 6.0);
    const real ft2 = Ct2 * std::exp(-Ct4 * ksi * ksi);
    n.A[I_NUT] = n.S[I_NUT] * n.U;
    n.B[I_NUT] = n.S[I_NUT] * n.V;
    const real Div_nu = (n.dkdx + n.dkdy);
    n.RX[I_NUT] = ((n.mu / n.S[I_RHO] + n.S[I_NUT]) * n.dkdx) / sig;
    n.RY[I_NUT] = ((n.mu / n.S[I_RHO] + n.S[I_NUT]) * n.dkdy) / sig;
    n.A[I_NUT] = n.A[I_NUT] - n.RX[I_NUT];
    n.B[I_NUT] = n.B[I_NUT] - n.RY[I_NUT];
    n.Src[I_NUT] = Cb1 * (1.0 - ft2) * S_hat * n.S[I_NUT] -
                   (Cw1 * fw - Cb1 / (_k * _k) * ft2) * (n.S[I_NUT] / n.l_min) * (n.S[I_NUT] / n.l_min) +
                   (Cb2 * Div_nu * Div_nu) / sig - C5 * nu_hat * nu_hat / a_sound2 * n.dUdy * n.dVdx;
  }
  turb_axisym_addon(n, P, is_init);
  if (is_mu_t) {
    n.mu_t = hf_max(0.0, (n.S[I_RHO] * n.S[I_NUT] * fv1));
    n.lam_t = n.mu_t * n.CP;
  }
}

// ---------------------------------------------------------------------------
// Turbulence closures.
// ---------------------------------------------------------------------------
// KEPS_ONLY: the caller guarantees that no node carries a model bit other
// than k-eps (lean N-S kernel), so only that branch is compiled in.
template <class N, bool KEPS_ONLY = false>
HF_HD inline void turb_model(N& n, const FillParams& P, int is_mu_t, int is_init) {
  const real dx = P.dx, dy = P.dy;
  real l = hf_max(n.l_min, hf_min(dy, dx)) * 0.41;
  const u64 TT = n.TurbType;
  if (!KEPS_ONLY && has_all(TT, TCT_Prandtl_Model)) {
    const real A_p = 26.0;
    const real n_0 = n.l_min * 0.41;
    if (P.tem == TEM_Prandtl) {
      l = n_0;
    } else if (P.tem == TEM_vanDriest) {
      l = n_0 * (1. - std::exp(-n.y_plus / A_p));
    } else if (P.tem == TEM_Escudier) {
      l = (P.delta > 0.) ? hf_min(n_0, 0.09 * P.delta) : n_0;
    } else if (P.tem == TEM_Klebanoff) {
      l = (P.delta > 0.) ? n_0 / std::sqrt(1 + 5.5 * powi_ref(n.l_min / P.delta, 6)) : n_0;
    }
    n.mu_t = n.S[I_RHO] * l * l * hf_max(std::fabs(n.dUdy), std::fabs(n.dVdx));
    n.lam_t = n.mu_t * n.CP;
  } else if (has_all(TT, TCT_k_eps_Model)) {
    real C1eps = 1.44, C2eps = 1.92, C_mu = 0.09, sig_k = 1.0, sig_eps = 1.3;
    real f1 = 1., f2 = 1., f_mu = 1.;
    real Rt, G, L_k = 0, L_eps = 0, Mt = 0;
    const real Tmp1 = n.dUdy + n.dVdx;
    const real Tmp2 = n.S[I_RHO] * l;
    real Tmp3 = n.dUdx * n.dUdx + n.dVdy * n.dVdy;
    if (P.FT) Tmp3 += hf_div(n.U, n.y);
    if (n.mu_t == 0) n.mu_t = n.S[I_RHO] * l * l * hf_max(std::fabs(n.dUdy), std::fabs(n.dVdx));
    G = n.mu_t * (Tmp1 * Tmp1 + 2 * Tmp3);
    if (n.S[I_EPS] != 0.0 && n.mu != 0.0)
      Rt = hf_div(hf_div(n.S[I_K] * n.S[I_K], n.S[I_EPS]), n.mu);
    else
      Rt = 0;
    if (P.tem == TEM_k_eps_Chien) {
      C1eps = 1.35;
      C2eps = 1.8;
      f2 = 1.0 - 0.4 / 1.8 * std::exp(-(Rt * Rt) / 36.0);
      f_mu = 1.0 - std::exp(-0.0115 * n.y_plus);
      L_k = -2.0 * n.mu * n.S[I_K] / (Tmp2 * Tmp2);
      L_eps = -2.0 * n.mu * n.S[I_EPS] / (Tmp2 * Tmp2) * std::exp(-n.y_plus / 2.0);
      Mt = 1.5 * n.S[I_K] / n.k / n.p;
    } else if (P.tem == TEM_k_eps_JL) {
      f_mu = std::exp(-2.5 / (1.0 + Rt / 50));
    } else if (P.tem == TEM_k_eps_LSY) {
      f_mu = std::exp(-3.4 / (1.0 + Rt / 50.0) / (1.0 + Rt / 50.0));
    } else if (P.tem == TEM_k_eps_RNG) {
      const real nu_0 = 4.38;
      real nu = (n.S[I_EPS] != 0.) ? std::sqrt(G) * n.S[I_K] / n.S[I_EPS] : 0;
      C_mu = 0.0845;
      C1eps = 1.42;
      C2eps = 1.68 + C_mu * nu * nu * nu * (1.0 - nu / nu_0) / (1. + 0.012 * nu * nu * nu);
      sig_k = 0.7194;
      sig_eps = 0.7194;
      f_mu = 1.;
    }
    if (is_init) {
      const real TmpI = P.turb_I * std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
      n.S[I_K] = 1.5 * TmpI * TmpI * n.S[I_RHO];
      n.S[I_EPS] = std::pow(C_mu, 3. / 4.) * std::pow(n.S[I_K] / n.S[I_RHO], 3. / 2.) / l;
      if (n.S[I_EPS] != 0)
        n.mu_t = std::fabs(C_mu * f_mu * n.S[I_K] * n.S[I_K] / n.S[I_EPS]);
    }
    if (has_all(TT, TCT_k_CONST)) {
      const real TmpI = P.turb_I * std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
      n.S[I_K] = 1.5 * TmpI * TmpI * n.S[I_RHO];
    }
    if (has_all(TT, TCT_eps_CONST))
      n.S[I_EPS] = std::pow(C_mu, 3. / 4.) * std::pow(n.S[I_K] / n.S[I_RHO], 3. / 2.) / l;
    if (has_all(TT, TCT_eps_Cmk2kXn_WALL))
      n.S[I_EPS] = std::pow(C_mu, 3. / 4.) * std::pow(n.S[I_K] / n.S[I_RHO], 3. / 2.) / l;
    if (is_mu_t && n.S[I_EPS] != 0) {
      const real nu_t = std::fabs(hf_div(C_mu * f_mu * n.S[I_K] * n.S[I_K], n.S[I_EPS]));
      n.mu_t = hf_min(nu_t, n.mu_t);
    }
    if (!is_init) {
      n.A[I_K] = n.S[I_K] * n.U;
      n.A[I_EPS] = n.S[I_EPS] * n.U;
      n.B[I_K] = n.S[I_K] * n.V;
      n.B[I_EPS] = n.S[I_EPS] * n.V;
      n.RX[I_K] = (n.mu + hf_div(n.mu_t, sig_k)) * (n.dkdx);
      n.RX[I_EPS] = (n.mu + hf_div(n.mu_t, sig_eps)) * (n.depsdx);
      n.RY[I_K] = (n.mu + hf_div(n.mu_t, sig_k)) * (n.dkdy);
      n.RY[I_EPS] = (n.mu + hf_div(n.mu_t, sig_eps)) * (n.depsdy);
      n.A[I_K] = n.A[I_K] - n.RX[I_K];
      n.A[I_EPS] = n.A[I_EPS] - n.RX[I_EPS];
      n.B[I_K] = n.B[I_K] - n.RY[I_K];
      n.B[I_EPS] = n.B[I_EPS] - n.RY[I_EPS];
      if (n.S[I_K] != 0.) {
        n.SrcAdd[I_K] = n.SrcAdd[I_EPS] = 0.;
        if (!has_all(TT, TCT_k_CONST))
          n.Src[I_K] = (G - n.S[I_EPS] * (1 + Mt) + L_k * n.S[I_RHO]);
        if (!has_all(TT, TCT_eps_CONST) && n.S[I_K] != 0)
          n.Src[I_EPS] = (hf_div(C1eps * f1 * n.S[I_EPS], n.S[I_K]) * G -
                          hf_div(C2eps * f2 * n.S[I_EPS] * n.S[I_EPS], n.S[I_K]) + L_eps * n.S[I_RHO]);
      }
      turb_axisym_addon(n, P, is_init);
    }
  } else if (!KEPS_ONLY && has_all(TT, TCT_Spalart_Allmaras_Model)) {
    turb_sa(n, P, is_mu_t, is_init);
  } else if (!KEPS_ONLY && has_all(TT, TCT_k_omega_SST_Model)) {
    turb_sst(n, P, is_mu_t, is_init);
  } else if (!KEPS_ONLY && has_all(TT, TCT_Integral_Model) && n.mu != 0.0) {
    n.Re_local = n.l_min *
                 std::sqrt(n.S[I_RHOU] * n.S[I_RHOU] + n.S[I_RHOV] * n.S[I_RHOV] + 1.e-30) / n.mu;
  } else if (!KEPS_ONLY && has_all(TT, TCT_Smagorinsky_Model)) {
    const real Cs = 0.1;
    const real _delta = std::sqrt(dx * dy);
    const real Wxy = 0.5 * (n.dVdx - n.dUdy);
    const real Omega = std::sqrt(2.0 * Wxy * Wxy);
    if (is_mu_t) {
      n.mu_t = hf_max(0.0, (n.S[I_RHO] * (Cs * _delta) * (Cs * _delta) * Omega));
      n.lam_t = n.mu_t * n.CP;
    }
  }
}

// ---------------------------------------------------------------------------
// FillNode2D equivalent.  Returns false when the node is skipped.
// ---------------------------------------------------------------------------
// Mixture closure of fill_node.  RefMix is the reference's: k = Cp/(Cp-R)
// from the previous step's mixture Cp and R, formation enthalpy sum Hu_i rhoY_i
// over the four species slots, p = (k-1)(rhoE - rho|V|^2/2 - H_f).  Mechanism
// mode (stepkern.hpp MechMix) replaces the three marked places.
struct RefMix {
  static constexpr bool MECH = false;
  template <class N>
  HF_HD void state(N&) const {}
  template <class N>
  HF_HD void heat_flux(const N&, real&, real&) const {}
};

// fill_node() in three pieces, so that the mechanism-mode lean step
// (hip/lean_mech.hpp) can run the part of a node that decides its thermodynamic
// state -- skip tests, velocity recovery, wall conditions, T by Newton -- once
// per cell (mech_state_node) and the flux part per tile and ring cell with that
// state loaded.  fill_node() calls them in this order, so both are the same
// arithmetic.
//   fill_node_pre   skip tests and U, V from the conserved momentum
//   (turbulence model)
//   fill_node_wall  wall-law / no-slip velocity and wall sources
template <class N>
HF_HD inline bool fill_node_pre(N& n) {
  if (has_all(n.CT, CT_SOLID)) return false;
  if (n.S[I_RHO] == 0) return false;
  if (n.k < 1) return false;
  // every branch writes both members (same values as "if U const: rho*U,
  // else U = rhoU/rho"): two stores to different members under a branch
  // are merged by the compiler into one store through a selected address,
  // which puts the whole node struct in scratch memory on the GPU
  const bool uc = has_all(n.CT, CT_U_CONST), vc = has_all(n.CT, CT_V_CONST);
  const real r = n.S[I_RHO], su = n.S[I_RHOU], sv = n.S[I_RHOV];
  const real u = uc ? n.U : hf_div(su, r), v = vc ? n.V : hf_div(sv, r);
  n.S[I_RHOU] = uc ? u * r : su;
  n.S[I_RHOV] = vc ? v * r : sv;
  n.U = u;
  n.V = v;
  return true;
}

template <class N>
HF_HD inline void fill_node_wall(N& n, const FillParams& P) {
  if (has_all(n.CT, CT_WALL_LAW)) {
    const real Tmp1 = std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
    n.S[I_RHOU] = Tmp1 * n.BGX;
    n.S[I_RHOV] = Tmp1 * n.BGY;
    n.U = n.S[I_RHOU] / n.S[I_RHO];
    n.V = n.S[I_RHOV] / n.S[I_RHO];
  } else if (has_all(n.CT, CT_WALL_NO_SLIP)) {
    n.U = n.S[I_RHOU] / n.S[I_RHO];
    n.V = n.S[I_RHOV] / n.S[I_RHO];
    if (P.isSrcAdd) {
      n.SrcAdd[I_RHO] = n.BGX * (n.U - n.Uw) * n.S[I_RHO] / P.dx + n.BGY * (n.V - n.Vw) * n.S[I_RHO] / P.dy;
      n.SrcAdd[I_RHOU] = n.BGX * (n.U - n.Uw) * n.S[I_RHO];
      n.SrcAdd[I_RHOV] = n.BGY * (n.V - n.Vw) * n.S[I_RHO];
      n.SrcAdd[I_RHOE] = 0.;
    } else {
      n.SrcAdd[I_RHOU] = n.SrcAdd[I_RHOV] = n.SrcAdd[I_RHOE] = 0.;
    }
    n.U = n.Uw;
    n.V = n.Vw;
    for (int i = 0; i < NCOMP; i++) n.SrcAdd[4 + i] = P.isSrcAdd ? n.SrcAdd[I_RHO] * n.Y[i] : 0.;
    n.S[I_RHOU] = n.U * n.S[I_RHO];
    n.S[I_RHOV] = n.V * n.S[I_RHO];
  } else {
    for (int i = 0; i < NEQ; i++) n.SrcAdd[i] = 0.;
  }
}

// TURB = 0: the caller guarantees that no node carries a turbulence-model
// bit (SK_SGL, lean.cpp sk_eligible), so turb_model() is a no-op and is not
// compiled in (its Spalart-Allmaras branch alone put the node in scratch);
// TURB = 2: k-eps is the only model bit present (lean N-S kernel);
// TURB = 3 / 4: k-omega SST / Spalart-Allmaras is the only one (lean steps).
template <class N, class MX = RefMix, int TURB = 1>   // TURB: 0 none, 1 every model, 2 k-eps, 3 SST, 4 SA only
HF_HD inline bool fill_node(N& n, const FillParams& P, const MX& mx = MX{}) {
  if (!fill_node_pre(n)) return false;
  real Tmp1, Tmp2 = 0, Tmp3 = 0., _mu = 0, _lam = 0, L = 0;
  if (!MX::MECH) n.k = hf_div(n.CP, n.CP - n.R);   // (k is not read by fill_node_pre's velocity part)

  if (P.sm == SM_NS) {
    if (P.is_init && n.TurbType > 0) {
      n.mu_t = 5.0 * n.mu;
    } else if (P.is_init) {
      n.mu_t = n.lam_t = 0.;
    }
    if (TURB == 3) {
      if (has_all(n.TurbType, TCT_k_omega_SST_Model)) turb_sst(n, P, P.is_mu_t, P.is_init);
    } else if (TURB == 4) {
      if (has_all(n.TurbType, TCT_Spalart_Allmaras_Model)) turb_sa(n, P, P.is_mu_t, P.is_init);
    } else if (TURB != 0 && n.TurbType > 0) {
      turb_model<N, TURB == 2>(n, P, P.is_mu_t, P.is_init);
    }
  }

  if (!MX::MECH) {
    Tmp1 = n.S[I_RHO];
    for (int i = 0; i < NCOMP; i++) {
      Tmp3 += P.Hu[i] * n.S[i + 4];
      Tmp1 -= n.S[i + 4];
    }
    Tmp3 += P.Hu[NCOMP] * Tmp1;
  }

  fill_node_wall(n, P);

  if (MX::MECH) {
    mx.state(n);   // T by Newton on the thermally perfect e(T); R, Cp, k, p at T
  } else {
    n.p = (n.k - 1.) * (n.S[I_RHOE] - n.S[I_RHO] * (n.U * n.U + n.V * n.V) * 0.5 - Tmp3);
    n.Tg = hf_div(hf_div(n.p, n.R), n.S[I_RHO]);
  }

  if (P.sm == SM_NS) {
    n.lam_t = n.mu_t * n.CP;
    if (P.is_mu_t) {
      if (has_all(n.CT, CT_WALL_NO_SLIP) || has_all(n.CT, CT_WALL_LAW)) {
        _mu = hf_max(0, (n.mu + n.mu_t * P.sig_w));
        _lam = hf_max(0, (n.lam + n.lam_t * P.sig_w));
      } else {
        _mu = hf_max(0, (n.mu + n.mu_t * P.sig_f));
        _lam = hf_max(0, (n.lam + n.lam_t * P.sig_f));
      }
    } else {
      _mu = n.mu;
      _lam = n.lam;
    }
    n.Diff = hf_div(_lam, n.CP);
    L = (2. / 3.) * _mu;
    if (P.FT == FT_AXISYMMETRIC)
      Tmp2 = L * (n.dUdx + n.dVdy + hf_div((real)P.FT * n.V, n.y));
    else
      Tmp2 = L * (n.dUdx + n.dVdy);
  }

  n.A[I_RHO] = n.S[I_RHOU];
  n.A[I_RHOU] = n.p + n.S[I_RHOU] * n.U;
  n.A[I_RHOV] = n.S[I_RHOV] * n.U;
  n.A[I_RHOE] = (n.S[I_RHOE] + n.p) * n.U;
  n.B[I_RHO] = n.S[I_RHOV];
  n.B[I_RHOU] = n.A[I_RHOV];
  n.B[I_RHOV] = n.p + n.S[I_RHOV] * n.V;
  n.B[I_RHOE] = (n.S[I_RHOE] + n.p) * n.V;
  for (int i = 4; i < 4 + NCOMP; i++) {
    n.B[i] = n.S[i] * n.V;
    n.A[i] = n.S[i] * n.U;
  }
  if (P.FT == FT_AXISYMMETRIC) {
    const real FT = (real)P.FT;
    n.F[I_RHO] = FT * n.B[I_RHO];
    n.F[I_RHOU] = FT * n.A[I_RHOV];
    n.F[I_RHOV] = FT * n.F[I_RHO] * n.V;
    n.F[I_RHOE] = FT * n.B[I_RHOE];
    for (int i = 4; i < 4 + NCOMP; i++) n.F[i] = FT * n.B[i];
  }
  if (P.sm == SM_NS) {
    const real sxx = 2. * _mu * n.dUdx - Tmp2;
    const real syy = 2. * _mu * n.dVdy - Tmp2;
    const real txy = _mu * (n.dUdy + n.dVdx);
    real qx = _lam * n.dTdx;
    real qy = _lam * n.dTdy;
    if (MX::MECH) {
      mx.heat_flux(n, qx, qy);   // sum_s Diff h_s(T) d(rho Y_s)
    } else {
      for (int i = 0; i < NSPEC; i++) {
        qx += n.Diff * (n.CP * n.Tg + P.Hu[i]) * n.droYdx[i];
        qy += n.Diff * (n.CP * n.Tg + P.Hu[i]) * n.droYdy[i];
      }
    }
    n.RX[I_RHO] = 0.;
    n.RX[I_RHOU] = sxx;
    n.RX[I_RHOV] = txy;
    n.RX[I_RHOE] = n.U * sxx + n.V * txy + qx;
    n.RY[I_RHO] = 0;
    n.RY[I_RHOU] = txy;
    n.RY[I_RHOV] = syy;
    n.RY[I_RHOE] = n.U * txy + n.V * syy + qy;
    n.A[I_RHOU] = n.A[I_RHOU] - n.RX[I_RHOU];
    n.A[I_RHOV] = n.A[I_RHOV] - n.RX[I_RHOV];
    n.A[I_RHOE] = n.A[I_RHOE] - n.RX[I_RHOE];
    n.B[I_RHOU] = n.B[I_RHOU] - n.RY[I_RHOU];
    n.B[I_RHOV] = n.B[I_RHOV] - n.RY[I_RHOV];
    n.B[I_RHOE] = n.B[I_RHOE] - n.RY[I_RHOE];
    for (int i = 4; i < 4 + NCOMP; i++) {
      n.RX[i] = n.Diff * n.droYdx[i - 4];
      n.RY[i] = n.Diff * n.droYdy[i - 4];
      n.A[i] = n.A[i] - n.RX[i];
      n.B[i] = n.B[i] - n.RY[i];
    }
    if (P.FT == FT_AXISYMMETRIC) {
      const real t00 = hf_div(2 * _mu * n.V, n.y) - Tmp2;
      n.F[I_RHOU] -= n.RY[I_RHOU];
      n.F[I_RHOV] -= n.RY[I_RHOV] + t00;
      n.F[I_RHOE] -= n.RY[I_RHOE];
      for (int i = 4; i < 4 + NCOMP; i++) n.F[i] -= n.RY[i];
    } else {
      for (int i = 0; i < NEQ; i++) n.F[i] = 0.;
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// Zeldovich "infinite-speed" global reaction + mixture properties.
// ---------------------------------------------------------------------------
template <class N>
HF_HD inline void chemistry_zeldovich(N& n, const SpeciesProps& sp, int sm, int model = CRM_ZELDOVICH) {
  real Yfu = n.S[I_YFU] / n.S[0];
  real Yox = n.S[I_YOX] / n.S[0];
  real Ycp = n.S[I_YCP] / n.S[0];
  real Yair = 1. - (Yfu + Yox + Ycp);
  real Y0;
  if (model == CRM_ZELDOVICH) {
    if (!has_all(n.CT, CT_Y_CONST)) {
      Y0 = 1. / (Yfu + Yox + Ycp + Yair);
      Yfu = Yfu * Y0;
      Yox = Yox * Y0;
      Ycp = Ycp * Y0;
      if (n.Tg > n.Tf) {
        if (Yox > Yfu * sp.K0) {
          Yox = Yox - Yfu * sp.K0;
          Yfu = 0.;
          Ycp = 1. - Yox - Yair;
        } else {
          Yfu = Yfu - Yox / sp.K0;
          Yox = 0.;
          Ycp = 1. - Yfu - Yair;
        }
      }
    }
  }
  const real T = n.Tg;
  n.R = sp.R[H_FU] * Yfu + sp.R[H_OX] * Yox + sp.R[H_CP] * Ycp + sp.R[H_AIR] * Yair;
  // mix(tables, Y): sum_s table_s(T) * Y_s.  A species with Y_s == 0
  // contributes +0 for any finite table value, so its table lookup is skipped
  // (identical result; saves the linear searches for single-gas flows).
  auto mix = [&](const TableData* t) {
    const real a = Yfu != 0 ? table_eval(t[H_FU], T) * Yfu : 0.;
    const real b = Yox != 0 ? table_eval(t[H_OX], T) * Yox : 0.;
    const real c = Ycp != 0 ? table_eval(t[H_CP], T) * Ycp : 0.;
    const real d = Yair != 0 ? table_eval(t[H_AIR], T) * Yair : 0.;
    return a + b + c + d;
  };
  n.CP = mix(sp.Cp);
  if (sm == SM_NS) {
    n.lam = mix(sp.lam);
    n.mu = mix(sp.mu);
  }
  if (Yair < 1.e-5) Yair = 0.;
  if (Ycp < 1.e-8) Ycp = 0.;
  if (Yox < 1.e-8) Yox = 0.;
  if (Yfu < 1.e-8) Yfu = 0.;
  Y0 = 1. / (Yfu + Yox + Ycp + Yair);
  Yfu = Yfu * Y0;
  Yox = Yox * Y0;
  Ycp = Ycp * Y0;
  Yair = Yair * Y0;
  n.Y[0] = Yfu;
  n.Y[1] = Yox;
  n.Y[2] = Ycp;
  n.Y[3] = Yair;
  if (!has_all(n.CT, CT_Y_CONST)) {
    n.S[I_YFU] = std::fabs(Yfu * n.S[0]);
    n.S[I_YOX] = std::fabs(Yox * n.S[0]);
    n.S[I_YCP] = std::fabs(Ycp * n.S[0]);
  }
}

// chemistry_zeldovich() for a viscous node whose fuel/oxidiser/product
// partial densities are +0: every zero-fraction term of the mixture sums is
// +0, so R = R_air, Cp/lam/mu = table_air(T) * 1 and Y = (0, 0, 0, 1) exactly
// (the species S stay +0).  Used by the single-gas laminar N-S path.
template <class N>
HF_HD inline void chemistry_single_gas_ns(N& n, const SpeciesProps& sp) {
  const real T = n.Tg;
  n.R = ((sp.R[H_FU] * 0. + sp.R[H_OX] * 0.) + sp.R[H_CP] * 0.) + sp.R[H_AIR] * 1.;
  n.CP = table_eval(sp.Cp[H_AIR], T) * 1.;
  n.lam = table_eval(sp.lam[H_AIR], T) * 1.;
  n.mu = table_eval(sp.mu[H_AIR], T) * 1.;
  n.Y[0] = n.Y[1] = n.Y[2] = 0.;
  n.Y[3] = 1.;
}

// Finite-rate global H2/air reaction (new; the reference declares the
// CRM_ARRENIUS slot without implementing it): 2 H2 + O2 -> 2 H2O with
// W = A exp(-Ta/T) [H2]^a [O2]^b (default: the one-step global rate with
// A = 1.8e13 (cm^3/mol)^0.5/s, E = 35 kcal/mol, a = 1, b = 0.5, in SI).
// The chemical energy is part of rho*E through the formation enthalpies
// (fill_node's Tmp3), so only species sources are needed; the product mass
// coefficient is (2 M_fu + M_ox) / 2 so mass is conserved exactly by
// construction.  One step may consume at most the available reactants.
template <class N>
HF_HD inline void chemistry_arrhenius_src(N& n, const SpeciesProps& sp, real dt) {
  const real T = n.Tg;
  const real Mfu = sp.M[H_FU], Mox = sp.M[H_OX];
  n.Src[I_YFU] = n.Src[I_YOX] = n.Src[I_YCP] = 0.;
  if (has_all(n.CT, CT_Y_CONST) || !(Mfu > 0) || !(Mox > 0) || !(T > 0)) return;
  const real cfu = n.S[I_YFU] / Mfu, cox = n.S[I_YOX] / Mox;   // mol/m^3
  if (!(cfu > 0) || !(cox > 0)) return;
  real W = sp.arr_A * std::exp(-sp.arr_Ta / T) * std::pow(cfu, sp.arr_a) * std::pow(cox, sp.arr_b);
  if (dt > 0) W = hf_min(W, hf_min(0.5 * cfu, cox) / dt);
  n.Src[I_YFU] = -2.0 * Mfu * W;
  n.Src[I_YOX] = -Mox * W;
  n.Src[I_YCP] = (2.0 * Mfu + Mox) * W;
}

// Number of transported equations for a cell: 9 for k-eps / SST (2 extra),
// 8 for Spalart-Allmaras, 7 otherwise (deeps2d_core.cpp:4683-4695).
HF_HD inline int num_eq_for(u64 turb_type) {
  if (has_all(turb_type, TCT_Prandtl_Model)) return NEQ - 2;
  if (has_all(turb_type, TCT_k_eps_Model)) return NEQ;
  if (has_all(turb_type, TCT_Spalart_Allmaras_Model)) return NEQ - 1;
  if (has_all(turb_type, TCT_k_omega_SST_Model)) return NEQ;
  return NEQ - 2;
}

HF_HD inline bool is_two_eq(u64 tt) {
  return has_all(tt, TCT_k_eps_Model) || has_all(tt, TCT_k_omega_SST_Model);
}
HF_HD inline bool has_turb_eq(u64 tt) {
  return has_all(tt, TCT_k_eps_Model) || has_all(tt, TCT_Spalart_Allmaras_Model) ||
         has_all(tt, TCT_k_omega_SST_Model);
}

}  // namespace hf2d
