// Detailed finite-rate chemistry: mechanism data, thermodynamics, transport and
// the point-implicit per-cell integrator (host + device).
//
// The reference reserves CRM_ARRENIUS / CRM_EDM (hyper_flow_bound.hpp:37-42) and
// hard-wires four species slots (NUM_COMPONENTS 3 + air, hyper_flow_node.hpp:
// 33-39).  In mechanism mode (deck ChemicalReactionsModel = 2 with a
// `Mechanism` key) the species of a detailed mechanism (<= 16, runtime count)
// are carried as extra conserved variables rho*Y_s next to the reference record
// (whose fuel/ox/cp slots stay zero), with
//   * a thermally perfect mixture: NASA-7 polynomials, e(T) = sum Y_s (h_s - R_s T)
//     including the formation enthalpies; T is recovered from rho*E by Newton
//     (replacing the reference's k = Cp/(Cp-R) closure, fill_node MechMix);
//   * mass-weighted transport (the reference's mixing rule) from Chapman-Enskog
//     species viscosities and Eucken conductivities, tabulated on a uniform T
//     grid (O(1) lookup) when the mechanism is loaded;
//   * operator-split kinetics: after each transport predictor the species of
//     every reacting cell are advanced over dt at constant (rho, e) by nsub
//     linearised backward-Euler substeps (I - h J) dc = h w(c, T), with the
//     analytic Jacobian J = N D, reversible rates from equilibrium constants,
//     third-body efficiencies and Troe fall-off, and T re-solved from e after
//     every substep.
// The bath gas (last species) is not transported: rho*Y_bath = rho - sum(others),
// like the reference's air remainder.
#pragma once

#include <cmath>

#include "common.hpp"

namespace hf2d {

constexpr int MECH_MAXSP = 16;
constexpr int MECH_MAXR = 64;
constexpr int MECH_MAXTB = 16;    // reactions with efficiency rows
constexpr int MECH_NT = 97;       // transport table: 200 K .. 5000 K, 50 K steps
constexpr real MECH_TT0 = 200.0, MECH_TDT = 50.0;
constexpr real MECH_RU = 8.314462618;
constexpr real MECH_PATM = 101325.0;
// Newton clamp.  Below MECH_TLO (the lower limit of the NASA-7 fits, 200 K
// for the GRI / Li et al. data) every species is extrapolated at constant cp
// -- cp(T) = cp(TLO), h(T) = h(TLO) + cp(TLO) (T - TLO), s(T) = s(TLO) +
// cp(TLO) ln(T / TLO) -- instead of running the polynomial outside its fit;
// the recovery then holds down to MECH_TMIN (reaching it flags the state as
// unphysical).  The under-expanded fuel jet of the scramjet deck cools to
// ~105 K in its barrel (profiles/scramjet_long_r05.md), so the former 100 K
// floor stopped that run after 12-14k steps.
constexpr real MECH_TMIN = 20.0, MECH_TMAX = 6000.0, MECH_TLO = 200.0;

struct MechReaction {
  int nrs = 0, nps = 0;            // distinct reactant / product species (<= 3 each)
  int rs[3] = {0, 0, 0}, rn[3] = {0, 0, 0};
  int ps[3] = {0, 0, 0}, pn[3] = {0, 0, 0};
  int rev = 1;                     // reverse rate from the equilibrium constant
  int tb = 0;                      // "+ M": rate multiplied by the collider concentration
  int fo = 0;                      // "(+M)": Lindemann / Troe fall-off
  int eff = -1;                    // row of MechData::eff (tb or fo), -1: all efficiencies 1
  int ntroe = 0;                   // 0 Lindemann, 3 or 4 Troe parameters
  int dnu = 0;                     // sum(nu'') - sum(nu')
  real A = 0, b = 0, Ta = 0;       // k (k_inf) = A T^b exp(-Ta / T), SI
  real A0 = 0, b0 = 0, Ta0 = 0;    // k_0 of a fall-off step
  real troe[4] = {0, 0, 0, 0};     // a, T3, T1, T2
};

struct MechData {
  int ns = 0, nr = 0, ntb = 0;
  int bath = 0;                    // remainder species (not transported)
  int nsub = 1;                    // point-implicit substeps per flow step
  real Tchem = 300.0;              // cells below this temperature do not react
  real W[MECH_MAXSP] = {};         // kg/mol
  real Rs[MECH_MAXSP] = {};        // RU / W
  real Tmid[MECH_MAXSP] = {};
  real a[MECH_MAXSP][2][7] = {};   // NASA-7 [low, high]
  real mu_tab[MECH_MAXSP][MECH_NT] = {};
  real lam_tab[MECH_MAXSP][MECH_NT] = {};
  real slot[4][MECH_MAXSP] = {};   // reference (fuel, ox, cp, air) -> species mass fractions
  int slot_sp[4] = {-1, -1, -1, -1};   // dominant species of each slot (Tecplot Y columns)
  real eff[MECH_MAXTB][MECH_MAXSP] = {};
  MechReaction rx[MECH_MAXR];
};

// ---------------------------------------------------------------------------
// Thermodynamics (per unit R: cp/R, h/(RT), s/R) and mixture relations
// ---------------------------------------------------------------------------
HF_HD inline const real* mech_coef(const MechData& m, int s, real T) { return m.a[s][T < m.Tmid[s] ? 0 : 1]; }
// The same coefficients as mech_coef() by value: both ranges are read at
// addresses that do not depend on T (on the GPU: scalar loads, issued ahead
// of the T-dependent arithmetic) and the range is picked per lane by a
// select.  Indexing with the T-dependent range made every species of every
// Newton iteration of mech_T_from_e a per-lane gather and a full memory round
// trip (the mechanism fill's T recovery was latency-bound on them).
struct Nasa7 {
  real a[7];
};
HF_HD inline Nasa7 mech_coef_v(const MechData& m, int s, real T) {
  const real* lo = m.a[s][0];
  const real* hi = m.a[s][1];
  const bool low = T < m.Tmid[s];
  Nasa7 c;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const real l = lo[k], h = hi[k];
    c.a[k] = low ? l : h;
  }
  return c;
}
HF_HD inline real nasa_cp(const real* a, real T) { return a[0] + T * (a[1] + T * (a[2] + T * (a[3] + T * a[4]))); }
HF_HD inline real nasa_h(const real* a, real T) {
  return a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2))) + a[5] / T;
}
// T * h/(RT) = T * (a0 + a1/2 T + ... + a4/5 T^4) + a5: the same polynomial
// without the division by T (the mixture energy and the species enthalpies
// need h, not h/RT; nine divisions per evaluation saved in the mechanism
// fill and in every Newton iteration of the temperature)
HF_HD inline real nasa_hT(const real* a, real T) {
  return T * (a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2)))) + a[5];
}
HF_HD inline real nasa_s(const real* a, real T, real lnT) {
  return a[0] * lnT + T * (a[1] + T * (a[2] * 0.5 + T * (a[3] * (1.0 / 3.0) + T * a[4] * 0.25))) + a[6];
}

// e (J/kg, formation included), cv, R_mix, cp of mass fractions Y at T
// (below MECH_TLO: evaluated at TLO, e extended linearly with the mixture cv
// -- the constant-cp extrapolation of every species; bitwise the polynomial
// for T >= TLO).
template <int NSB>
HF_HD inline void mech_mix_thermo(const MechData& m, const real* Y, real T, real* e, real* cv, real* Rm, real* cp) {
  real se = 0, scv = 0, sR = 0;
  const real Te = T < MECH_TLO ? MECH_TLO : T;
#pragma unroll
  for (int s = 0; s < NSB; s++) {
    if (s >= m.ns) break;
    const Nasa7 c = mech_coef_v(m, s, Te);
    const real* a = c.a;
    const real R = m.Rs[s];
    se += Y[s] * R * (nasa_hT(a, Te) - Te);
    scv += Y[s] * R * (nasa_cp(a, Te) - 1.0);
    sR += Y[s] * R;
  }
  se += scv * (T - Te);   // (+0 for T >= TLO: branch-free, the fill kernels are sensitive to code shape)
  *e = se;
  *cv = scv;
  *Rm = sR;
  *cp = scv + sR;
}

// Temperature from the specific internal energy by Newton iteration (T0: guess).
template <int NSB>
HF_HD inline real mech_T_from_e(const MechData& m, const real* Y, real e, real T0) {
  real T = T0 > MECH_TMIN ? (T0 < MECH_TMAX ? T0 : MECH_TMAX) : MECH_TMIN;
  for (int it = 0; it < 30; it++) {
    real ee, cv, R, cp;
    mech_mix_thermo<NSB>(m, Y, T, &ee, &cv, &R, &cp);
    real dT = (e - ee) / cv;
    if (dT > 500.0) dT = 500.0;
    if (dT < -500.0) dT = -500.0;
    real Tn = T + dT;
    Tn = Tn > MECH_TMIN ? (Tn < MECH_TMAX ? Tn : MECH_TMAX) : MECH_TMIN;
    const real d = Tn - T;
    T = Tn;
    if (std::fabs(d) <= 1e-10 * T) break;
  }
  return T;
}

// Mass-weighted mixture viscosity / conductivity (uniform-grid tables).
template <int NSB>
HF_HD inline void mech_transport(const MechData& m, const real* Y, real T, real* mu, real* lam) {
  real x = (T - MECH_TT0) * (1.0 / MECH_TDT);
  int i = (int)x;
  if (x < 0) i = 0;
  if (i > MECH_NT - 2) i = MECH_NT - 2;
  const real w = x - (real)i;   // linear inter/extrapolation from the end segments
  real smu = 0, slam = 0;
  // the per-lane table reads of every species first (s < NSB <= MECH_MAXSP
  // rows always exist), then the sums of the mechanism's species in order:
  // one memory round trip instead of one per species
  static_assert(NSB <= MECH_MAXSP, "species block larger than the tables");
  real m0[NSB], m1[NSB], l0[NSB], l1[NSB];
#pragma unroll
  for (int s = 0; s < NSB; s++) {
    m0[s] = m.mu_tab[s][i];
    m1[s] = m.mu_tab[s][i + 1];
    l0[s] = m.lam_tab[s][i];
    l1[s] = m.lam_tab[s][i + 1];
  }
  // (predicated, not `break`: a runtime trip count makes the compiler roll
  // the loop and index the register arrays dynamically, through scratch)
#pragma unroll
  for (int s = 0; s < NSB; s++) {
    if (s < m.ns) {
      smu += Y[s] * (m0[s] + (m1[s] - m0[s]) * w);
      slam += Y[s] * (l0[s] + (l1[s] - l0[s]) * w);
    }
  }
  *mu = smu;
  *lam = slam;
}

// Species absolute enthalpy h_s(T) (J/kg) for the enthalpy-diffusion heat flux.
HF_HD inline real mech_h_species(const MechData& m, int s, real T) {
  const real Te = T < MECH_TLO ? MECH_TLO : T;
  const Nasa7 c = mech_coef_v(m, s, Te);
  // constant cp below TLO, branch-free (+0 above it): a branch here made the
  // lean mechanism tile kernel 7 % slower; cp(TLO) from the coefficients in
  // registers (a per-species table load cost the tile kernel 2 VGPR spills)
  return m.Rs[s] * (nasa_hT(c.a, Te) + nasa_cp(c.a, Te) * (T - Te));
}

// ---------------------------------------------------------------------------
// Kinetics: rate constants of one reaction at T (kf incl. fall-off, kr) and the
// net rate of progress / its concentration derivatives.
// ---------------------------------------------------------------------------
HF_HD inline real ipow3(real x, int n) { return n == 1 ? x : (n == 2 ? x * x : (n == 3 ? x * x * x : 1.0)); }

struct MechRate {
  real kf, kr, mult, dM;   // dM: 1 if d(mult)/dc_j = eff_j (pure third body), else 0
};

// g[s] = h_s/(R T) - s_s/R of every species at T (for equilibrium constants)
// (below MECH_TLO with the constant-cp extrapolation: h/RT = (h(TLO)/R +
// cp/R (T - TLO)) / T, s/R = s(TLO)/R + cp/R ln(T / TLO))
template <int NSB>
HF_HD inline void mech_gibbs(const MechData& m, real T, real lnT, real* g) {
  const bool lo = T < MECH_TLO;
  const real Te = lo ? MECH_TLO : T;
  const real lnTe = lo ? std::log(MECH_TLO) : lnT;
#pragma unroll
  for (int s = 0; s < NSB; s++) {
    if (s >= m.ns) break;
    const Nasa7 c = mech_coef_v(m, s, Te);
    if (lo) {
      const real cpR = nasa_cp(c.a, Te);
      g[s] = (nasa_hT(c.a, Te) + cpR * (T - Te)) / T - (nasa_s(c.a, Te, lnTe) + cpR * (lnT - lnTe));
    } else {
      g[s] = nasa_h(c.a, T) - nasa_s(c.a, T, lnT);
    }
  }
}

HF_HD inline MechRate mech_rate(const MechData& m, const MechReaction& r, const real* g, const real* c, real T,
                                real lnT, real invT, real lnP0RT) {
  MechRate q;
  real kf = r.A * std::exp(r.b * lnT - r.Ta * invT);
  real M = 1.0;
  if (r.tb || r.fo) {
    M = 0.0;
    if (r.eff >= 0) {
      for (int s = 0; s < m.ns; s++) M += m.eff[r.eff][s] * c[s];
    } else {
      for (int s = 0; s < m.ns; s++) M += c[s];
    }
  }
  q.dM = 0.0;
  if (r.fo) {
    const real k0 = r.A0 * std::exp(r.b0 * lnT - r.Ta0 * invT);
    const real Pr = k0 * M / kf;
    real F = 1.0;
    if (r.ntroe >= 3) {
      real Fc = (1.0 - r.troe[0]) * std::exp(-T / r.troe[1]) + r.troe[0] * std::exp(-T / r.troe[2]);
      if (r.ntroe > 3) Fc += std::exp(-r.troe[3] * invT);
      const real lFc = std::log10(Fc > 1e-300 ? Fc : 1e-300);
      const real lPr = std::log10(Pr > 1e-300 ? Pr : 1e-300);
      const real cc = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;
      const real f1 = (lPr + cc) / (nn - 0.14 * (lPr + cc));
      F = std::pow(10.0, lFc / (1.0 + f1 * f1));
    }
    kf = kf * (Pr / (1.0 + Pr)) * F;
    q.mult = 1.0;
  } else {
    q.mult = M;
    q.dM = r.tb ? 1.0 : 0.0;
  }
  q.kf = kf;
  if (r.rev) {
    real sg = 0;
    for (int t = 0; t < r.nps; t++) sg += r.pn[t] * g[r.ps[t]];
    for (int t = 0; t < r.nrs; t++) sg -= r.rn[t] * g[r.rs[t]];
    // ln Kc = -sum nu g + dnu ln(P0 / (RU T));  kr = kf / Kc
    const real lnKc = -sg + r.dnu * lnP0RT;
    q.kr = kf * std::exp(-lnKc);
  } else {
    q.kr = 0.0;
  }
  return q;
}

// One point-implicit (linearised backward-Euler) chemistry update of a cell at
// constant density and internal energy.  rhoY: species partial densities (in /
// out), T: temperature guess in, final temperature out.  Runtime mechanism
// data (any mechanism <= NSB species); the host reference of the device
// kernels (chem_fast.hip for compiled mechanisms, chem_mech.hip MFMA for
// runtime ones).  Returns false if the linear system was singular.
template <int NSB>
HF_HD inline bool mech_chem_cell(const MechData& m, real rho, real e, real* rhoY, real* T, real dt, int nsub) {
  const int ns = m.ns;
  real c[NSB], Y[NSB], g[NSB], om[NSB], J[NSB][NSB];
  for (int s = 0; s < ns; s++) {
    c[s] = rhoY[s] > 0 ? rhoY[s] / m.W[s] : 0.0;
    Y[s] = c[s] * m.W[s] / rho;
  }
  real Tc = mech_T_from_e<NSB>(m, Y, e, *T);
  const real h = dt / nsub;
  bool ok = true;
  for (int sub = 0; sub < nsub; sub++) {
    const real lnT = std::log(Tc), invT = 1.0 / Tc;
    const real lnP0RT = std::log(MECH_PATM / (MECH_RU * Tc));
    mech_gibbs<NSB>(m, Tc, lnT, g);
    for (int i = 0; i < ns; i++) {
      om[i] = 0;
      for (int j = 0; j < ns; j++) J[i][j] = 0;
    }
    for (int ir = 0; ir < m.nr; ir++) {
      const MechReaction& r = m.rx[ir];
      const MechRate k = mech_rate(m, r, g, c, Tc, lnT, invT, lnP0RT);
      real pf = 1.0, pr = 1.0;
      for (int t = 0; t < r.nrs; t++) pf *= ipow3(c[r.rs[t]], r.rn[t]);
      for (int t = 0; t < r.nps; t++) pr *= ipow3(c[r.ps[t]], r.pn[t]);
      const real net = k.kf * pf - k.kr * pr;
      const real q = k.mult * net;
      for (int t = 0; t < r.nrs; t++) om[r.rs[t]] -= r.rn[t] * q;
      for (int t = 0; t < r.nps; t++) om[r.ps[t]] += r.pn[t] * q;
      // D_j = dq/dc_j for every species touching the step
      real D[NSB];
      for (int j = 0; j < ns; j++) D[j] = 0;
      for (int t = 0; t < r.nrs; t++) {
        real d = k.kf * r.rn[t] * ipow3(c[r.rs[t]], r.rn[t] - 1);
        for (int u = 0; u < r.nrs; u++)
          if (u != t) d *= ipow3(c[r.rs[u]], r.rn[u]);
        D[r.rs[t]] += k.mult * d;
      }
      for (int t = 0; t < r.nps; t++) {
        real d = k.kr * r.pn[t] * ipow3(c[r.ps[t]], r.pn[t] - 1);
        for (int u = 0; u < r.nps; u++)
          if (u != t) d *= ipow3(c[r.ps[u]], r.pn[u]);
        D[r.ps[t]] -= k.mult * d;
      }
      if (k.dM != 0.0)
        for (int j = 0; j < ns; j++) D[j] += (r.eff >= 0 ? m.eff[r.eff][j] : 1.0) * net;
      for (int t = 0; t < r.nrs; t++)
        for (int j = 0; j < ns; j++) J[r.rs[t]][j] -= r.rn[t] * D[j];
      for (int t = 0; t < r.nps; t++)
        for (int j = 0; j < ns; j++) J[r.ps[t]][j] += r.pn[t] * D[j];
    }
    // (I - h J) dc = h om : Gaussian elimination with partial pivoting
    real Mx[NSB][NSB + 1];
    for (int i = 0; i < ns; i++) {
      for (int j = 0; j < ns; j++) Mx[i][j] = (i == j ? 1.0 : 0.0) - h * J[i][j];
      Mx[i][ns] = h * om[i];
    }
    for (int k = 0; k < ns; k++) {
      int p = k;
      real best = std::fabs(Mx[k][k]);
      for (int i = k + 1; i < ns; i++)
        if (std::fabs(Mx[i][k]) > best) {
          best = std::fabs(Mx[i][k]);
          p = i;
        }
      if (!(best > 0.0)) {
        ok = false;
        break;
      }
      if (p != k)
        for (int j = k; j <= ns; j++) {
          const real t = Mx[k][j];
          Mx[k][j] = Mx[p][j];
          Mx[p][j] = t;
        }
      const real inv = 1.0 / Mx[k][k];
      for (int i = k + 1; i < ns; i++) {
        const real f = Mx[i][k] * inv;
        if (f != 0.0)
          for (int j = k; j <= ns; j++) Mx[i][j] -= f * Mx[k][j];
      }
    }
    if (!ok) break;
    for (int i = ns - 1; i >= 0; i--) {
      real s = Mx[i][ns];
      for (int j = i + 1; j < ns; j++) s -= Mx[i][j] * om[j];
      om[i] = s / Mx[i][i];   // om now holds dc
    }
    real tot = 0;
    for (int s = 0; s < ns; s++) {
      c[s] = c[s] + om[s];
      if (c[s] < 0) c[s] = 0;
      tot += c[s] * m.W[s];
    }
    // restore sum(rho Y) = rho (clipping removes mass)
    const real sc = tot > 0 ? rho / tot : 1.0;
    for (int s = 0; s < ns; s++) {
      c[s] *= sc;
      Y[s] = c[s] * m.W[s] / rho;
    }
    Tc = mech_T_from_e<NSB>(m, Y, e, Tc);
  }
  for (int s = 0; s < ns; s++) rhoY[s] = c[s] * m.W[s];
  *T = Tc;
  return ok;
}

}  // namespace hf2d
