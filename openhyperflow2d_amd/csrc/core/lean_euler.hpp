// Lean inviscid step: predictor + FillNode2D + chemistry of one cell in a
// single pass, with the neighbour fluxes recomputed from their state instead
// of loaded.
//
// The generic Jacobi stepper (stepkern.hpp) keeps the reference's per-node
// record alive in SoA form: A, B, F, Src, SrcAdd, p, k, R, CP, Tg, ... are
// re-read and re-written every step (~2 KB of HBM traffic per cell-step).
// For an inviscid case without gas sources the inviscid fluxes of a node
// (FillNode2D flux block, reference libFlow FlowNode2D.hpp FillNode2D) are a
// pure function of
//   S[0..3] (committed), the pre-chemistry species S[4..6] and U, V, p
// of that node's last fill, so the persistent per-cell state shrinks to
//   S (7), Spre (3), beta (7), U, V, p, CP, R  (+ Y, Tg, k written for output)
// plus dS/dx, dS/dy on the few nodes a Cauchy (d2/dx2 = 0) neighbour reads.
// Every value is produced by the same expressions as fill_node(),
// chemistry_zeldovich() and predict_core(), so the lean path equals the
// generic stepper bit for bit.  The device solver switches freely between
// the two: the first lean step after a generic one reads the generic A/B/F
// (FROM_GENERIC), and lean_materialize_cell() rebuilds A/B/F/p before any
// generic step.
//
// Single-gas specialisation (SG): when every node's fuel/oxidiser/product
// partial densities are +0 (air-only decks: all the reference test cases),
// they stay +0 bit for bit under predictor, fill and Zeldovich chemistry (the
// species fluxes are +-0, the LxF update yields +0, chemistry maps Y to
// (0,0,0,1) and stores fabs(0 * rho)), so the species equations, their
// pre-chemistry copies and betas need not be touched at all; the mixture
// terms reduce to R = R_air, Cp = Cp_air(T).  lean_single_gas() checks it.
//
// Eligibility (lean_eligible() on the host): inviscid, no gas sources,
// adiabatic walls, Src == 0 everywhere, SrcAdd == 0 except on no-slip nodes
// (whose SrcAdd lives in its array), every non-solid node set.
#pragma once

#include <algorithm>
#include <cstring>

#include "stepkern.hpp"

namespace hf2d {

// the two doubles have the same bits (+0 / -0 and NaNs told apart)
HF_HD inline bool same_bits(real a, real b) {
  u64 x, y;
  std::memcpy(&x, &a, sizeof x);
  std::memcpy(&y, &b, sizeof y);
  return x == y;
}

// per-cell lean byte: neighbour bits (NB_*) | who must publish dS/dx, dS/dy
// LB_PLAIN: interior node on the flag-free predictor fast path (predict_core
// PLAIN) -- set on the host by lean_flags().
enum : uint8_t { LB_DX_OUT = 16, LB_DY_OUT = 32, LB_PLAIN = 64 };

struct LeanSoA {
  long N = 0;
  const real* Sin;     // [NEQ*N] committed state (equations 0..6 used)
  real* Sout;
  const real* Pin_s;   // [NCOMP*N] pre-chemistry species of the last fill
  real* Pout_s;
  real* beta;          // in place
  const real* Uin;
  const real* Vin;
  const real* Pin;     // pressure (FROM_GENERIC: the generic p array)
  real* Uout;
  real* Vout;
  real* Pout;
  real* Tout;          // Tg of this fill (output only for Euler)
  const real* dSdx_in;
  const real* dSdy_in;
  real* dSdx_out;
  real* dSdy_out;
  const u64* CT;
  const uint8_t* lb;
  real* CP;            // in place (chemistry)
  real* R;             // in place (chemistry)
  real* kk;            // written (output)
  real* Y;             // [NSPEC*N] in place
  const real* Tf;
  const real* BGX;
  const real* BGY;
  real* SrcAdd;        // no-slip nodes only
  // FROM_GENERIC: the previous step was generic; use its flux arrays
  const real* gA;
  const real* gB;
  const real* gF;
};

// Inviscid fluxes of equation k at node `at` (fill_node's A/B assembly);
// species use the pre-chemistry partial densities.
HF_HD inline real lean_flux_A(const LeanSoA& L, int k, long at, real u, real p) {
  const long N = L.N;
  switch (k) {
    case I_RHO: return L.Sin[N + at];
    case I_RHOU: return p + L.Sin[N + at] * u;
    case I_RHOV: return L.Sin[2 * N + at] * u;
    case I_RHOE: return (L.Sin[3 * N + at] + p) * u;
    default: return L.Pin_s[(k - 4) * N + at] * u;
  }
}
HF_HD inline real lean_flux_B(const LeanSoA& L, int k, long at, real u, real v, real p) {
  const long N = L.N;
  switch (k) {
    case I_RHO: return L.Sin[2 * N + at];
    case I_RHOU: return L.Sin[2 * N + at] * u;
    case I_RHOV: return p + L.Sin[2 * N + at] * v;
    case I_RHOE: return (L.Sin[3 * N + at] + p) * v;
    default: return L.Pin_s[(k - 4) * N + at] * v;
  }
}

// The node's own per-step inputs that live in global memory, loaded up front
// (the tiled kernel issues these loads before its LDS barrier).
struct LeanOwn {
  u64 CT = 0;
  uint8_t lb = 0;
  bool filled = false;   // set and not solid
  real beta[4 + NCOMP];
  real CP = 0, R = 0, kk = 0;
};

// (Issuing these loads unconditionally instead -- no wait for CT -- measured
// ~4% slower on the headline grid: solid cells then load too.)
template <int NE = 4 + NCOMP>
HF_HD inline void lean_load_own(const LeanSoA& L, long idx, LeanOwn& o) {
  const long N = L.N;
  o.CT = L.CT[idx];
  o.lb = L.lb[idx];
  o.filled = !has_all(o.CT, CT_SOLID) && has_all(o.CT, CT_NODE_IS_SET);
  if (o.filled) {
#pragma unroll
    for (int k = 0; k < NE; k++) o.beta[k] = L.beta[k * N + idx];
    o.CP = L.CP[idx];
    o.R = L.R[idx];
    o.kk = L.kk[idx];
  }
}

// Accessor members shared by the global-memory and the LDS-tile IO: the
// node's own persistent arrays (beta, dS/dx, dS/dy, SrcAdd) stay in global
// memory, addressed by the global indices idx / iL / iR / iU / iD.
struct LeanIOCommon {
  static constexpr int NE = 4 + NCOMP;
  static constexpr bool skip(int) { return false; }
  HF_HD static constexpr int eq(int k) { return k; }
  const LeanSoA& L;
  long N, idx, iL, iR, iU, iD;
  uint8_t lb = 0;
  bool noslip = false;
  real FT = 0;
  const real* obeta = nullptr;   // LeanOwn::beta
  bool skip_same = false;        // StepParams::skip_same
  real sm[NEQ];

  HF_HD LeanIOCommon(const LeanSoA& l, long i) : L(l), N(l.N), idx(i), iL(i), iR(i), iU(i), iD(i) {}
  HF_HD void set_nb_global(int i, int j, int ny, int n1, int n2, int n3, int n4) {
    iL = (long)(i - n1) * ny + j;
    iR = (long)(i + n2) * ny + j;
    iU = idx + n3;
    iD = idx - n4;
  }
  HF_HD real dxL(int k) const { return L.dSdx_in[k * N + iL]; }
  HF_HD real dxR(int k) const { return L.dSdx_in[k * N + iR]; }
  HF_HD real dyU(int k) const { return L.dSdy_in[k * N + iU]; }
  HF_HD real dyD(int k) const { return L.dSdy_in[k * N + iD]; }
  HF_HD real beta(int k) const { return obeta[k]; }
  HF_HD real Src(int) const { return 0.0; }
  HF_HD real SrcAdd(int k) const { return noslip ? L.SrcAdd[k * N + idx] : 0.0; }
  HF_HD void put_S(int k, real v) { sm[k] = v; }
  HF_HD void put_beta(int k, real v) const {
    if (!skip_same || !same_bits(v, obeta[k])) L.beta[k * N + idx] = v;
  }
  HF_HD void put_dS(int k, real a, real b) const {
    if (lb & LB_DX_OUT) L.dSdx_out[k * N + idx] = a;
    if (lb & LB_DY_OUT) L.dSdy_out[k * N + idx] = b;
  }
  HF_HD void keep_dS(int k) const {
    if (lb & LB_DX_OUT) L.dSdx_out[k * N + idx] = L.dSdx_in[k * N + idx];
    if (lb & LB_DY_OUT) L.dSdy_out[k * N + idx] = L.dSdy_in[k * N + idx];
  }
  // the node's new lean state (the persistent kernel keeps it on chip)
  HF_HD void out_S(int k, real v) const { L.Sout[k * N + idx] = v; }
  HF_HD void out_Ps(int k, real v) const { L.Pout_s[k * N + idx] = v; }
  HF_HD void out_UVP(real u, real v, real p) const {
    L.Uout[idx] = u;
    L.Vout[idx] = v;
    L.Pout[idx] = p;
  }
  HF_HD void out_CP(real v) const { L.CP[idx] = v; }
  HF_HD void out_R(real v) const { L.R[idx] = v; }
};

// Global-memory IO.  FROMG: the previous step was generic, read its A/B/F.
template <bool FROMG>
struct LeanIO : LeanIOCommon {
  real uL, pL, uR, pR, uU, vU, pU, uD, vD, pD, u0, v0, p0;

  HF_HD LeanIO(const LeanSoA& l, long i) : LeanIOCommon(l, i) {
    u0 = L.Uin[idx];
    v0 = L.Vin[idx];
    p0 = L.Pin[idx];
  }
  HF_HD real U0() const { return u0; }
  HF_HD real V0() const { return v0; }
  HF_HD real P0() const { return p0; }
  HF_HD void set_nb(int i, int j, int ny, int n1, int n2, int n3, int n4) {
    set_nb_global(i, j, ny, n1, n2, n3, n4);
    if (!FROMG) {
      uL = L.Uin[iL];
      pL = L.Pin[iL];
      uR = L.Uin[iR];
      pR = L.Pin[iR];
      uU = L.Uin[iU];
      vU = L.Vin[iU];
      pU = L.Pin[iU];
      uD = L.Uin[iD];
      vD = L.Vin[iD];
      pD = L.Pin[iD];
    }
  }
  HF_HD real S(int k) const { return L.Sin[k * N + idx]; }
  HF_HD real SL(int k) const { return L.Sin[k * N + iL]; }
  HF_HD real SR(int k) const { return L.Sin[k * N + iR]; }
  HF_HD real SU(int k) const { return L.Sin[k * N + iU]; }
  HF_HD real SD(int k) const { return L.Sin[k * N + iD]; }
  HF_HD real AL(int k) const { return FROMG ? L.gA[k * N + iL] : lean_flux_A(L, k, iL, uL, pL); }
  HF_HD real AR(int k) const { return FROMG ? L.gA[k * N + iR] : lean_flux_A(L, k, iR, uR, pR); }
  HF_HD real BU(int k) const { return FROMG ? L.gB[k * N + iU] : lean_flux_B(L, k, iU, uU, vU, pU); }
  HF_HD real BD(int k) const { return FROMG ? L.gB[k * N + iD] : lean_flux_B(L, k, iD, uD, vD, pD); }
  // axisymmetric source of the node's own previous fill (fill_node F block)
  HF_HD real F(int k) const {
    if (FROMG) return L.gF[k * N + idx];
    switch (k) {
      case I_RHO: return FT * L.Sin[2 * N + idx];
      case I_RHOU: return FT * (L.Sin[2 * N + idx] * u0);
      case I_RHOV: return FT * (FT * L.Sin[2 * N + idx]) * v0;
      case I_RHOE: return FT * ((L.Sin[3 * N + idx] + p0) * v0);
      default: return FT * (L.Pin_s[(k - 4) * N + idx] * v0);
    }
  }
};

// Node as seen by chemistry_zeldovich().
struct LeanChemNode {
  real S[NEQ];
  real Tg, Tf, R, CP, lam, mu;
  real Y[NSPEC];
  u64 CT;
};

// chemistry_zeldovich() evaluated for a node whose species partial densities
// are +0: Y = (0, 0, 0, 1), R = R_air, Cp = Cp_air(T) (each zero-fraction term
// of the mixture sums is +0, so the sums reduce to the air term exactly).
// (A copy of the air Cp table in the kernel arguments, scanned branch-free,
// cost 95 SGPR spills in the tile kernel and ~9 % of its time: measured and
// removed.)
template <class N>
HF_HD inline void chemistry_single_gas(N& n, const SpeciesProps& sp) {
  n.R = ((sp.R[H_FU] * 0. + sp.R[H_OX] * 0.) + sp.R[H_CP] * 0.) + sp.R[H_AIR] * 1.;
  n.CP = table_eval(sp.Cp[H_AIR], n.Tg) * 1.;
  n.Y[0] = n.Y[1] = n.Y[2] = 0.;
  n.Y[3] = 1.;
}

// One lean step of cell (i, j) through accessor `io` (constructed on idx).
// Returns the local dt limit (1.0 if none).
// OUT: also write the output-only fields (Tg, k, Y); the solver requests them
// on the last step before control returns to the host (downloads, outputs).
template <bool RES, bool OUT, class IO>
HF_HD inline real lean_cell(const StepParams& P, const LeanSoA& L, IO& io, const LeanOwn& own, int i, int j,
                            ResidualPack& res, int* neg_T) {
  const long N = L.N;
  const long idx = io.idx;
  const u64 CT = own.CT;
  const uint8_t lb = own.lb;
  constexpr int NE = IO::NE;              // transported equations touched
  constexpr bool SG = IO::NE == 4;        // single-gas specialisation
  io.lb = lb;
  io.obeta = own.beta;
  io.skip_same = P.skip_same != 0;
  if (!own.filled) {
    // neither transported nor filled: carry the state into the other buffers
    for (int k = 0; k < NE; k++) io.out_S(k, io.S(k));
    if (lb & (LB_DX_OUT | LB_DY_OUT))
      for (int k = 0; k < NEQ; k++) io.keep_dS(k);
    return 1.0;
  }
  const bool active = !has_all(CT, NT_FC);
  const bool noslip = has_all(CT, CT_WALL_NO_SLIP);
  io.noslip = noslip;
  io.FT = (real)P.fpa.FT;
  const real u_old = io.U0(), v_old = io.V0();
  if (active) {
    const int n1 = (lb & NB_XL) ? 1 : 0, n2 = (lb & NB_XR) ? 1 : 0;
    const int n3 = (lb & NB_YU) ? 1 : 0, n4 = (lb & NB_YD) ? 1 : 0;
    io.set_nb(i, j, P.ny, n1, n2, n3, n4);
    // Equations >= NE are frozen for inviscid cells: TurbType only matters
    // through num_eq_for(), which is >= NE for every model.
    if (lb & LB_PLAIN)
      predict_core<RES, IO, true>(P, io, CT, (u64)0, n1, n2, n3, n4, P.gx0 + i, j, res);
    else
      predict_core<RES, IO, false>(P, io, CT, (u64)0, n1, n2, n3, n4, P.gx0 + i, j, res);
    if (lb & (LB_DX_OUT | LB_DY_OUT))
      for (int k = NE; k < NEQ; k++) io.keep_dS(k);
  } else {
    for (int k = 0; k < NE; k++) io.sm[k] = io.S(k);
    if (lb & (LB_DX_OUT | LB_DY_OUT))
      for (int k = 0; k < NEQ; k++) io.keep_dS(k);
  }

  // ---- FillNode2D, inviscid subset (fill_node) ----
  LeanChemNode c;
  for (int k = 0; k < NE; k++) c.S[k] = io.sm[k];
  for (int k = NE; k < NEQ; k++) c.S[k] = 0.;
  real* s = c.S;
  // NT_FC nodes are filled with FillNode2D(1, 0, ...) (P.ffc): it differs
  // from P.fpa only in is_mu_t / is_init, which the inviscid fill never reads.
  // (A runtime-selected reference into the kernel-argument block would force
  // a scratch copy of StepParams.)
  const FillParams& F = P.fpa;
  c.R = own.R;
  c.CP = own.CP;
  const real k_old = own.kk;
  if (s[I_RHO] == 0 || k_old < 1) {
    // fill_node() skipped the node: keep the previous primitives
    for (int k = 0; k < NE; k++) io.out_S(k, s[k]);
    if (!SG)
      for (int k = 0; k < NCOMP; k++) io.out_Ps(k, s[4 + k]);
    io.out_UVP(u_old, v_old, io.P0());
    return 1.0;
  }
  const real kk = hf_div(c.CP, c.CP - c.R);
  real U, V;
  if (has_all(CT, CT_U_CONST)) {
    U = u_old;
    s[I_RHOU] = U * s[I_RHO];
  } else {
    U = hf_div(s[I_RHOU], s[I_RHO]);
  }
  if (has_all(CT, CT_V_CONST)) {
    V = v_old;
    s[I_RHOV] = V * s[I_RHO];
  } else {
    V = hf_div(s[I_RHOV], s[I_RHO]);
  }
  real Tmp1 = s[I_RHO], Tmp3 = 0.;
  for (int q = 0; q < NCOMP; q++) {
    Tmp3 += F.Hu[q] * s[q + 4];
    Tmp1 -= s[q + 4];
  }
  Tmp3 += F.Hu[NCOMP] * Tmp1;
  if (has_all(CT, CT_WALL_LAW)) {
    Tmp1 = std::sqrt(U * U + V * V + 1.e-30);
    s[I_RHOU] = Tmp1 * L.BGX[idx];
    s[I_RHOV] = Tmp1 * L.BGY[idx];
    U = s[I_RHOU] / s[I_RHO];
    V = s[I_RHOV] / s[I_RHO];
  } else if (noslip) {
    U = s[I_RHOU] / s[I_RHO];
    V = s[I_RHOV] / s[I_RHO];
    real* sa = L.SrcAdd;
    const real Uw = 0.0, Vw = 0.0;
    if (F.isSrcAdd) {
      const real bgx = L.BGX[idx], bgy = L.BGY[idx];
      sa[I_RHO * N + idx] = bgx * (U - Uw) * s[I_RHO] / F.dx + bgy * (V - Vw) * s[I_RHO] / F.dy;
      sa[I_RHOU * N + idx] = bgx * (U - Uw) * s[I_RHO];
      sa[I_RHOV * N + idx] = bgy * (V - Vw) * s[I_RHO];
      sa[I_RHOE * N + idx] = 0.;
    } else {
      sa[I_RHOU * N + idx] = sa[I_RHOV * N + idx] = sa[I_RHOE * N + idx] = 0.;
    }
    U = Uw;
    V = Vw;
    for (int q = 0; q < NCOMP; q++)
      sa[(4 + q) * N + idx] = F.isSrcAdd ? sa[I_RHO * N + idx] * L.Y[q * N + idx] : 0.;
    s[I_RHOU] = U * s[I_RHO];
    s[I_RHOV] = V * s[I_RHO];
  }
  const real p = (kk - 1.) * (s[I_RHOE] - s[I_RHO] * (U * U + V * V) * 0.5 - Tmp3);
  const real Tg = hf_div(hf_div(p, c.R), s[I_RHO]);
  // fluxes of this fill are built from the pre-chemistry species
  if (!SG)
    for (int k = 0; k < NCOMP; k++) io.out_Ps(k, s[4 + k]);
  real dt_local = 1.0;
  if (active) {
    if (Tg < 0.) {
      if (neg_T) *neg_T = 1;
    } else {
      const real AAA = hf_sqrt(kk * c.R * Tg);
      dt_local = P.CFL_min * hf_min(hf_div(P.dx, AAA + std::fabs(U)), hf_div(P.dy, AAA + std::fabs(V)));
      if (P.chem_model != NO_REACTIONS) {
        c.Tg = Tg;
        c.Tf = L.Tf[idx];
        c.CT = CT;
        c.lam = c.mu = 0.;
        if (SG)
          chemistry_single_gas(c, *P.species);
        else
          chemistry_zeldovich(c, *P.species, P.sm, P.chem_model);
        if (c.R != own.R) io.out_R(c.R);   // constant for a frozen mixture
        if (!io.skip_same || !same_bits(c.CP, own.CP)) io.out_CP(c.CP);
        // Y is output-only except for the no-slip SrcAdd of the next step
        if (OUT || noslip)
          for (int q = 0; q < NSPEC; q++) L.Y[q * N + idx] = c.Y[q];
      }
    }
  }
  for (int k = 0; k < NE; k++) io.out_S(k, s[k]);
  io.out_UVP(U, V, p);
  if (OUT) {
    L.Tout[idx] = Tg;
    L.kk[idx] = kk;
  }
  return dt_local;
}

// ---------------------------------------------------------------------------
// LDS-tiled form.  A workgroup owns a TI x TJ tile of cells (TJ along the
// contiguous j axis, sized so ny splits into equal tiles of <= 64) and first
// stages the tile plus its one-cell cross-shaped halo -- S (7), pre-chemistry
// species (3), U, V, p -- into LDS with independent coalesced loads; every
// neighbour flux is then evaluated from LDS.  The node's own beta / CP / R /
// k / flags come straight from global memory (read once).
// ---------------------------------------------------------------------------
constexpr int LEAN_TILE_FIELDS = 13;   // S[0..6], Spre[0..2], U, V, p
constexpr int LEAN_TILE_FIELDS_SG = 7; // single gas: S[0..3], U, V, p
inline int lean_tile_fields(bool sg) { return sg ? LEAN_TILE_FIELDS_SG : LEAN_TILE_FIELDS; }
constexpr int LEAN_TILE_MIN_TJ = 8;

struct LeanTile {
  int TI, TJ, W, NC, nbi, nbj;
  int TIh;   // columns per cell layer: thread t owns (t / TJ + q * TIh, t % TJ), q < CPT
  int CPT;   // cells per thread
  // comm-overlap launches: tile columns at the strip's right edge in the edge
  // part (2 when the last one holds a single column and the halo carries two)
  int ne = 1;
};

// Tile height: tj > 0 overrides (clamped to [LEAN_TILE_MIN_TJ, block]);
// otherwise the height in [16, 32] that wastes the fewest lanes and rows
// (measured: ~25-row tiles beat 50-row ones on 2000x200 by ~5%).
inline LeanTile lean_tile_geom(int ncols, int ny, int block, int tj = 0, int cpt = 1) {
  LeanTile T;
  if (tj > 0) {
    T.TJ = std::min(std::max(tj, LEAN_TILE_MIN_TJ), std::min(block, ny));
  } else if (ny <= 32) {
    T.TJ = ny;
  } else {
    double best = -1;
    T.TJ = 32;
    for (int c = 16; c <= 32; c++) {
      const int nj = (ny + c - 1) / c;
      const double eff = (double)((block / c) * c) / block * (double)ny / (nj * c);
      if (eff > best + 1e-12) {
        best = eff;
        T.TJ = c;
      }
    }
  }
  T.CPT = cpt;
  T.TIh = block / T.TJ;
  T.TI = T.TIh * cpt;
  T.W = T.TJ + 2;
  T.NC = (T.TI + 2) * T.W;
  T.nbi = (ncols + T.TI - 1) / T.TI;
  T.nbj = (ny + T.TJ - 1) / T.TJ;
  return T;
}

// Thread t of nthreads stages its share of tile (i0, j0).  LDS layout:
// lds[f * NC + c], c = (ii + 1) * W + (jj + 1), ii in [-1, TI], jj in [-1, TJ].
template <bool SG = false>
HF_HD inline void lean_tile_stage(const StepParams& P, const LeanSoA& L, const LeanTile& T, int i0, int j0,
                                  real* lds, int t, int nthreads) {
  const long N = L.N;
  const int NC = T.NC;
  constexpr int NS = SG ? 4 : 4 + NCOMP;          // staged state equations
  constexpr int FU = SG ? 4 : 10;                 // U, V, p field slots
  // (stepping the slot's (ii, jj) without the division per slot measured
  // 1.3 % slower on the headline grid, profiles/exchange_loopback_r05.md)
  for (int c = t; c < NC; c += nthreads) {
    const int ii = c / T.W - 1, jj = c - (ii + 1) * T.W - 1;
    const bool xh = ii < 0 || ii >= T.TI, yh = jj < 0 || jj >= T.TJ;
    const int gi = i0 + ii, gj = j0 + jj;
    if ((xh && yh) || gi < 0 || gi >= P.nx || gj < 0 || gj >= P.ny) continue;
    const long g = (long)gi * P.ny + gj;
#pragma unroll
    for (int f = 0; f < NS; f++) lds[f * NC + c] = L.Sin[f * N + g];
    if (!SG)
#pragma unroll
      for (int f = 0; f < NCOMP; f++) lds[(4 + NCOMP + f) * NC + c] = L.Pin_s[f * N + g];
    lds[FU * NC + c] = L.Uin[g];
    lds[(FU + 1) * NC + c] = L.Vin[g];
    lds[(FU + 2) * NC + c] = L.Pin[g];
  }
}

template <bool SG = false>
struct TileIO : LeanIOCommon {
  static constexpr int NE = SG ? 4 : 4 + NCOMP;
  static constexpr int FU = SG ? 4 : 10, FV = FU + 1, FP = FU + 2;
  const real* lds;
  int NC, W, c, cL, cR, cU, cD;

  HF_HD TileIO(const LeanSoA& l, long i, const real* s, int nc, int w, int cc)
      : LeanIOCommon(l, i), lds(s), NC(nc), W(w), c(cc), cL(cc), cR(cc), cU(cc), cD(cc) {}
  HF_HD real at(int f, int cc) const { return lds[f * NC + cc]; }
  HF_HD real U0() const { return at(FU, c); }
  HF_HD real V0() const { return at(FV, c); }
  HF_HD real P0() const { return at(FP, c); }
  HF_HD void set_nb(int i, int j, int ny, int n1, int n2, int n3, int n4) {
    set_nb_global(i, j, ny, n1, n2, n3, n4);
    cL = c - n1 * W;
    cR = c + n2 * W;
    cU = c + n3;
    cD = c - n4;
  }
  HF_HD real S(int k) const { return at(k, c); }
  HF_HD real SL(int k) const { return at(k, cL); }
  HF_HD real SR(int k) const { return at(k, cR); }
  HF_HD real SU(int k) const { return at(k, cU); }
  HF_HD real SD(int k) const { return at(k, cD); }
  HF_HD real fA(int k, int cc) const {
    const real u = at(FU, cc), p = at(FP, cc);
    switch (k) {
      case I_RHO: return at(1, cc);
      case I_RHOU: return p + at(1, cc) * u;
      case I_RHOV: return at(2, cc) * u;
      case I_RHOE: return (at(3, cc) + p) * u;
      default: return at(k + 3, cc) * u;
    }
  }
  HF_HD real fB(int k, int cc) const {
    const real u = at(FU, cc), v = at(FV, cc), p = at(FP, cc);
    switch (k) {
      case I_RHO: return at(2, cc);
      case I_RHOU: return at(2, cc) * u;
      case I_RHOV: return p + at(2, cc) * v;
      case I_RHOE: return (at(3, cc) + p) * v;
      default: return at(k + 3, cc) * v;
    }
  }
  HF_HD real AL(int k) const { return fA(k, cL); }
  HF_HD real AR(int k) const { return fA(k, cR); }
  HF_HD real BU(int k) const { return fB(k, cU); }
  HF_HD real BD(int k) const { return fB(k, cD); }
  HF_HD real F(int k) const {
    const real u0 = U0(), v0 = V0(), p0 = P0();
    switch (k) {
      case I_RHO: return FT * at(2, c);
      case I_RHOU: return FT * (at(2, c) * u0);
      case I_RHOV: return FT * (FT * at(2, c)) * v0;
      case I_RHOE: return FT * ((at(3, c) + p0) * v0);
      default: return FT * (at(k + 3, c) * v0);
    }
  }
};


// Logical tile b -> cell layer q of thread t; returns false for idle threads.
HF_HD inline bool lean_tile_cell(const StepParams& P, const LeanTile& T, int b, int t, int* i, int* j, int* c,
                                 int* i0, int* j0, int q = 0) {
  const int bi = b / T.nbj, bj = b - bi * T.nbj;
  *i0 = P.i0 + bi * T.TI;
  *j0 = bj * T.TJ;
  const int r = t / T.TJ, jj = t - r * T.TJ;
  const int ii = r + q * T.TIh;
  if (r >= T.TIh) {
    *i = *j = *c = 0;
    return false;
  }
  *i = *i0 + ii;
  *j = *j0 + jj;
  *c = (ii + 1) * T.W + jj + 1;
  return ii < T.TI && *i < P.i1 && *j < P.ny;
}

template <bool RES, bool FROMG>
HF_HD inline real lean_euler_cell(const StepParams& P, const LeanSoA& L, int i, int j, ResidualPack& res,
                                  int* neg_T) {
  const long idx = (long)i * P.ny + j;
  LeanOwn own;
  lean_load_own(L, idx, own);
  LeanIO<FROMG> io(L, idx);
  return lean_cell<RES, true>(P, L, io, own, i, j, res, neg_T);
}

// host convenience: nullable residual pack
template <class IO>
inline real lean_cell_host(const StepParams& P, const LeanSoA& L, IO& io, int i, int j, ResidualPack* res,
                           int* neg_T) {
  LeanOwn own;
  lean_load_own<IO::NE>(L, io.idx, own);
  if (res) return lean_cell<true, true>(P, L, io, own, i, j, *res, neg_T);
  ResidualPack d;
  return lean_cell<false, true>(P, L, io, own, i, j, d, neg_T);
}

// Rebuild the generic per-node fluxes (A, B, F) and p from the lean state,
// exactly as the last fill produced them.
HF_HD inline void lean_materialize_cell(const StepParams& P, const LeanSoA& L, const SoA& g, int i, int j) {
  const long N = L.N;
  const long idx = (long)i * P.ny + j;
  const u64 CT = L.CT[idx];
  if (has_all(CT, CT_SOLID) || !has_all(CT, CT_NODE_IS_SET)) return;
  const real U = L.Uin[idx], V = L.Vin[idx], p = L.Pin[idx];
  g.p[idx] = p;
  if (L.Sin[idx] == 0) return;
  constexpr int NE = 4 + NCOMP;
  for (int k = 0; k < NE; k++) {
    g.A[k * N + idx] = lean_flux_A(L, k, idx, U, p);
    g.B[k * N + idx] = lean_flux_B(L, k, idx, U, V, p);
  }
  if (P.fpa.FT == FT_AXISYMMETRIC) {
    const real FT = (real)P.fpa.FT;
    const real F0 = FT * L.Sin[2 * N + idx];
    g.F[idx] = F0;
    g.F[N + idx] = FT * (L.Sin[2 * N + idx] * U);
    g.F[2 * N + idx] = FT * F0 * V;
    g.F[3 * N + idx] = FT * ((L.Sin[3 * N + idx] + p) * V);
    for (int k = 4; k < NE; k++) g.F[k * N + idx] = FT * (L.Pin_s[(k - 4) * N + idx] * V);
  }
}

}  // namespace hf2d
