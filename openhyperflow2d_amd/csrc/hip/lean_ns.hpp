// Lean viscous step (single-gas N-S, SK_SGL): one LDS-tiled kernel per time
// step instead of the split predict + fill pair, with the fluxes of the
// step recomputed inside the tile instead of stored.
//
// Split stepper (stepkern.hpp), step n:
//   predict_n   S^n (committed), A^n, B^n (stored by the last fill), dt_n
//               -> Sp^{n+1} (predicted state), beta
//   fill_{n+1}  Sp^{n+1}, neighbours' Sp^{n+1} (rho gradient), the previous
//               fill's primitives P^n (U, V, T gradients; CP, mu, lam, k)
//               -> committed S^{n+1}, A/B^{n+1}, P^{n+1}, dt_{n+1}
// The fluxes A/B of every cell are a pure function of Sp and P of that cell
// and its four neighbours (reference FillNode2D, hyper_flow_node.hpp:373-600,
// called per cell at deeps2d_core.cpp:1169-1244), so they need not move
// through memory.  Kernel K_n of this path:
//   1. F_n (fill_compute, the same function the split fill runs) for the
//      tile's cells and its one-cell cross-shaped ring, from Sp^n and the
//      level n-1 primitives in global memory -> committed S^n, A^n, B^n into
//      LDS; the tile's own cells also store their level-n primitives;
//   2. predict_n (predict_core) of the tile's cells from LDS -> Sp^{n+1};
//   3. the own-cell part of F_{n+1} that dt_{n+1} needs (U, V, T, k of the
//      new state; no neighbours) -> dt_{n+1}.
// Persistent state per cell: Sp (4), beta (4), U/V/T and CP/mu/lam/k at two
// levels (ping-pong), i.e. ~270 B of HBM traffic per cell-step instead of
// ~460 B for the split pair; every value is produced by the same expressions
// as the split kernels, so the two paths are bitwise equal (GPU tests).  The
// device solver switches freely between them (DeviceSolver::lns_*).
#pragma once

#include "../core/lean_euler.hpp"

namespace hf2d {

// Kernel argument block.  Level m-1 = the primitives the fill F_m reads
// (prim_old of the split fill), level m = the ones it produces.
struct LnsArrays {
  long N = 0;
  const real* Sp = nullptr;   // Sp^m [k * N + idx] (live equations)
  real* Sp_out = nullptr;     // Sp^{m+1}
  real* beta = nullptr;       // in place
  const real *Ui = nullptr, *Vi = nullptr, *Ti = nullptr;
  real *Uo = nullptr, *Vo = nullptr, *To = nullptr;
  const real *CPi = nullptr, *mui = nullptr, *lami = nullptr, *kki = nullptr, *mu_ti = nullptr;
  real *CPo = nullptr, *muo = nullptr, *lamo = nullptr, *kko = nullptr, *mu_to = nullptr;
  const real *R = nullptr, *BGX = nullptr, *BGY = nullptr, *grad = nullptr, *l_min = nullptr, *y_plus = nullptr;
  // in place (a ring evaluation of another tile discards these outputs, so
  // only the owner's read-before-write matters)
  real* SrcAdd = nullptr;
  real* Src = nullptr;
  // generic fluxes: the turbulence equations' of a node without a k-eps
  // model bit are never rewritten by the fill (constant while lean)
  const real *gA = nullptr, *gB = nullptr, *gF = nullptr;
  const real* dSdx_in = nullptr;
  const real* dSdy_in = nullptr;
  real* dSdx_out = nullptr;
  real* dSdy_out = nullptr;
  const u64* CT = nullptr;
  const u64* TT = nullptr;
  const uint8_t* nb = nullptr;
  const uint8_t* gf = nullptr;
};

// live equations: SGL 0..3; SGT 0..3 + k, eps (LDS plane q(k))
template <int MODE>
struct Lns {
  static constexpr int NL = MODE == SK_SGT ? 6 : 4;
  static constexpr int PLANES = 3 * NL;   // committed S, A, B per LDS cell
  HF_HD static constexpr int q(int k) { return k < 4 ? k : k - 3; }
  HF_HD static constexpr int eqk(int qq) { return qq < 4 ? qq : qq + 3; }
};
constexpr int LNS_NL = 4;

// fill_compute() input accessor over the lean buffers (F_m of any cell of
// the tile or its ring).  Every input the fill reads is loaded up front in
// one batch -- the four neighbours' rho (and k, eps), U, V, T too, at
// clamped indices, selected by the neighbour bits later (a missing
// neighbour resolves to the cell itself, as in FillSoAIO) -- so a fill costs
// one memory latency instead of a chain of dependent ones.  Inputs the fill
// rewrites before any use (p, Diff, lam_t; k-eps: the k/eps fluxes) return
// +0; wall / inactive-only fields load on demand.
// TURB: fill_node's turbulence-model set of the SGT kernel (2 k-eps, 3 SST, 4
// Spalart-Allmaras; physics.hpp)
template <int MODE, int TURB = 2>
struct LnsFillIO {
  static constexpr int TURB_SET = TURB;
  static constexpr bool T2 = MODE == SK_SGT;
  static constexpr int NL = Lns<MODE>::NL;
  const LnsArrays& a;
  long N, idx;
  u64 ct, tt;
  uint8_t g, b;
  real s[NL], u, v, t, cp, mu_, lam_, kk_, r_, mut_, lmin_, yp_;
  real rn[4], un[4], vn[4], tn[4], kn[T2 ? 4 : 1], en[T2 ? 4 : 1];
  int nbit[4];
  HF_HD LnsFillIO(const LnsArrays& aa, int i, int j, int nx, int ny) : a(aa), N(aa.N), idx((long)i * ny + j) {
    const long nbi[4] = {i > 0 ? idx - ny : idx, i < nx - 1 ? idx + ny : idx, j < ny - 1 ? idx + 1 : idx,
                         j > 0 ? idx - 1 : idx};
    ct = a.CT[idx];
    tt = a.TT[idx];
    g = a.gf[idx];
    b = a.nb[idx];
#pragma unroll
    for (int q = 0; q < NL; q++) s[q] = a.Sp[Lns<MODE>::eqk(q) * N + idx];
    u = a.Ui[idx];
    v = a.Vi[idx];
    t = a.Ti[idx];
    cp = a.CPi[idx];
    mu_ = a.mui[idx];
    lam_ = a.lami[idx];
    kk_ = a.kki[idx];
    r_ = a.R[idx];
    if (T2) {
      mut_ = a.mu_ti[idx];
      lmin_ = a.l_min[idx];
      yp_ = a.y_plus[idx];
    } else {
      mut_ = lmin_ = yp_ = 0.0;
    }
#pragma unroll
    for (int d = 0; d < 4; d++) {
      rn[d] = a.Sp[nbi[d]];
      un[d] = a.Ui[nbi[d]];
      vn[d] = a.Vi[nbi[d]];
      tn[d] = a.Ti[nbi[d]];
      if (T2) {
        kn[T2 ? d : 0] = a.Sp[(long)I_K * N + nbi[d]];
        en[T2 ? d : 0] = a.Sp[(long)I_EPS * N + nbi[d]];
      }
      nbit[d] = 0;
    }
  }
  HF_HD void set_nb(int, int, int, int n1, int n2, int n3, int n4) {
    nbit[ND_L] = n1;
    nbit[ND_R] = n2;
    nbit[ND_U] = n3;
    nbit[ND_D] = n4;
  }
  // the turbulence fluxes fill_node rewrites on every node of the model (SA
  // leaves them on walls / NT_FC nodes: loaded)
  HF_HD bool keps() const {
    return (TURB == 2 && has_all(tt, TCT_k_eps_Model)) || (TURB == 3 && has_all(tt, TCT_k_omega_SST_Model));
  }
  HF_HD u64 CT() const { return ct; }
  HF_HD u64 TT() const { return tt; }
  HF_HD uint8_t gf() const { return g; }
  HF_HD uint8_t nb() const { return b; }
  HF_HD real S(int k) const { return s[Lns<MODE>::q(k)]; }
  HF_HD real Sn(int k, int d) const {
    if (k == 0) return nbit[d] ? rn[d] : s[0];
    if (T2 && k == I_K) return nbit[d] ? kn[T2 ? d : 0] : s[4];
    if (T2 && k == I_EPS) return nbit[d] ? en[T2 ? d : 0] : s[5];
    return 0.0;
  }
  // loaded only for the turbulence equations (fill_compute, in-place fluxes)
  HF_HD real A(int k) const { return keps() ? 0.0 : a.gA[k * N + idx]; }
  HF_HD real B(int k) const { return keps() ? 0.0 : a.gB[k * N + idx]; }
  HF_HD real F(int k) const { return keps() ? 0.0 : a.gF[k * N + idx]; }
  HF_HD real Src(int k) const { return a.Src[k * N + idx]; }
  HF_HD real SrcAdd(int k) const { return a.SrcAdd[k * N + idx]; }
  HF_HD real Uo() const { return u; }
  HF_HD real Vo() const { return v; }
  HF_HD real To() const { return t; }
  HF_HD real Uon(int d) const { return nbit[d] ? un[d] : u; }
  HF_HD real Von(int d) const { return nbit[d] ? vn[d] : v; }
  HF_HD real Ton(int d) const { return nbit[d] ? tn[d] : t; }
  HF_HD real p() const { return 0.0; }   // rewritten by fill_node before any use (no Chien model)
  HF_HD real kk() const { return kk_; }
  HF_HD real R() const { return r_; }
  HF_HD real CP() const { return cp; }
  HF_HD real lam() const { return lam_; }
  HF_HD real mu() const { return mu_; }
  HF_HD real Diff() const { return 0.0; }
  HF_HD real mu_t() const { return mut_; }
  HF_HD real lam_t() const { return 0.0; }
  HF_HD real l_min() const { return lmin_; }
  HF_HD real y_plus() const { return yp_; }
  HF_HD real Re_local() const { return 0.0; }
  HF_HD real BGX() const { return a.BGX[idx]; }
  HF_HD real BGY() const { return a.BGY[idx]; }
  HF_HD real Tf() const { return 0.0; }
  HF_HD real Y(int) const { return 0.0; }
  HF_HD real grad(int gg) const { return a.grad[gg * N + idx]; }
  HF_HD real Ys(int) const { return 0.0; }
  HF_HD real Ysn(int, int) const { return 0.0; }
};

// The node's level-m values kept in registers between F_m and the partial
// F_{m+1} (the split fill's prim_old / per-cell inputs of the next fill),
// plus its own F_m outputs the predictor reads (F, Src, SrcAdd).
template <int MODE>
struct LnsLevel {
  static constexpr int NL = Lns<MODE>::NL;
  real U, V, Tg, p, k, R, CP, lam, mu, mu_t, l_min, y_plus, BGX, BGY;
  real SrcAdd[NL], F[NL], Src[NL];
};

// Input accessor of the own-cell part of F_{m+1}: the new predicted state
// (registers) and the level-m values of the node (no neighbours: they only
// enter the fluxes, gradients and turbulence sources, which this part does
// not produce; dt needs U, V, T, k -- lns_eligible excludes a viscous CFL
// with an eddy viscosity).
template <int MODE>
struct LnsOwnIO {
  static constexpr int TURB_SET = 0;   // dt does not depend on the turbulence model
  const real* sn;   // Sp^{m+1} by equation index
  const LnsLevel<MODE>& v;
  u64 ct, tt;
  uint8_t g, b;
  HF_HD LnsOwnIO(const real* s, const LnsLevel<MODE>& lv, u64 c, u64 t, uint8_t gg, uint8_t bb)
      : sn(s), v(lv), ct(c), tt(t), g(gg), b(bb) {}
  HF_HD void set_nb(int, int, int, int, int, int, int) {}
  HF_HD u64 CT() const { return ct; }
  HF_HD u64 TT() const { return tt; }
  HF_HD uint8_t gf() const { return g; }
  HF_HD uint8_t nb() const { return b; }
  HF_HD real S(int k) const { return sn[k]; }
  HF_HD real Sn(int k, int) const { return sn[k]; }
  HF_HD real A(int) const { return 0.0; }
  HF_HD real B(int) const { return 0.0; }
  HF_HD real F(int) const { return 0.0; }
  HF_HD real Src(int k) const { return v.Src[Lns<MODE>::q(k)]; }
  HF_HD real SrcAdd(int k) const { return v.SrcAdd[Lns<MODE>::q(k)]; }
  HF_HD real Uo() const { return v.U; }
  HF_HD real Vo() const { return v.V; }
  HF_HD real To() const { return v.Tg; }
  HF_HD real Uon(int) const { return v.U; }
  HF_HD real Von(int) const { return v.V; }
  HF_HD real Ton(int) const { return v.Tg; }
  HF_HD real p() const { return v.p; }
  HF_HD real kk() const { return v.k; }
  HF_HD real R() const { return v.R; }
  HF_HD real CP() const { return v.CP; }
  HF_HD real lam() const { return v.lam; }
  HF_HD real mu() const { return v.mu; }
  HF_HD real Diff() const { return 0.0; }
  HF_HD real mu_t() const { return v.mu_t; }
  HF_HD real lam_t() const { return 0.0; }
  HF_HD real l_min() const { return v.l_min; }
  HF_HD real y_plus() const { return v.y_plus; }
  HF_HD real Re_local() const { return 0.0; }
  HF_HD real BGX() const { return v.BGX; }
  HF_HD real BGY() const { return v.BGY; }
  HF_HD real Tf() const { return 0.0; }
  HF_HD real Y(int) const { return 0.0; }
  HF_HD real grad(int) const { return 0.0; }
  HF_HD real Ys(int) const { return 0.0; }
  HF_HD real Ysn(int, int) const { return 0.0; }
};

// predict_core() accessor: committed S and the fluxes of the cell and its
// neighbours from LDS, the node's own F/Src/SrcAdd from registers (its F_m),
// beta and the Cauchy dS/dx, dS/dy in global memory.
template <int MODE>
struct LnsPredictIO {
  static constexpr int NL = Lns<MODE>::NL;
  static constexpr int NE = MODE == SK_SGL ? 4 : NEQ;
  static constexpr bool skip(int k) { return !sk_live(MODE, k); }
  HF_HD static constexpr int eq(int k) { return k; }
  const LnsArrays& a;
  const real* lds;
  const LnsLevel<MODE>& lv;
  const real* bpre;   // the node's beta, loaded before the tile barrier
  long N, idx, iL, iR, iU, iD;
  int NC, c, cL, cR, cU, cD;
  uint8_t gf;
  real sn[NEQ];
  HF_HD real at(int f, int cc) const { return lds[f * NC + cc]; }
  HF_HD static constexpr int q(int k) { return Lns<MODE>::q(k); }
  HF_HD real S(int k) const { return at(q(k), c); }
  HF_HD real SL(int k) const { return at(q(k), cL); }
  HF_HD real SR(int k) const { return at(q(k), cR); }
  HF_HD real SU(int k) const { return at(q(k), cU); }
  HF_HD real SD(int k) const { return at(q(k), cD); }
  HF_HD real AL(int k) const { return at(NL + q(k), cL); }
  HF_HD real AR(int k) const { return at(NL + q(k), cR); }
  HF_HD real BU(int k) const { return at(2 * NL + q(k), cU); }
  HF_HD real BD(int k) const { return at(2 * NL + q(k), cD); }
  HF_HD real dxL(int k) const { return a.dSdx_in[k * N + iL]; }
  HF_HD real dxR(int k) const { return a.dSdx_in[k * N + iR]; }
  HF_HD real dyU(int k) const { return a.dSdy_in[k * N + iU]; }
  HF_HD real dyD(int k) const { return a.dSdy_in[k * N + iD]; }
  HF_HD real beta(int k) const { return bpre[q(k)]; }
  HF_HD real F(int k) const { return lv.F[q(k)]; }
  // SoAPredictIO: the turbulence sources always, flow sources never (lns_ok)
  HF_HD real Src(int k) const { return k >= 4 + NCOMP ? lv.Src[q(k)] : 0.0; }
  HF_HD real SrcAdd(int k) const { return (gf & GF_SRCADD) ? lv.SrcAdd[q(k)] : 0.0; }
  HF_HD void put_S(int k, real v) { sn[k] = v; }
  HF_HD void put_beta(int k, real v) const { a.beta[k * N + idx] = v; }
  HF_HD void put_dS(int k, real x, real y) const {
    if (gf & GF_DX_OUT) a.dSdx_out[k * N + idx] = x;
    if (gf & GF_DY_OUT) a.dSdy_out[k * N + idx] = y;
  }
  HF_HD void keep_dS(int k) const {
    if (gf & GF_DX_OUT) a.dSdx_out[k * N + idx] = a.dSdx_in[k * N + idx];
    if (gf & GF_DY_OUT) a.dSdy_out[k * N + idx] = a.dSdy_in[k * N + idx];
  }
};

// Tile height of the lean N-S kernel (256 threads, one cell each): every
// wavefront evaluates its cells' fills, the ring cells take extra wavefront
// rounds, so minimise (own waves + ring waves) per useful cell over the
// heights that leave no partial tile row pattern too wasteful.
inline int lns_tile_height(int ny, int block) {
  int best = 16;
  double best_cost = 1e30;
  for (int c = LEAN_TILE_MIN_TJ; c <= 64 && c <= ny; c++) {
    const int ti = block / c, own = ti * c, ring = 2 * (ti + c);
    const int nj = (ny + c - 1) / c;
    const double eff = (double)ny / (nj * c);
    const double cost = (double)((own + 63) / 64 + (ring + 63) / 64) / (own * eff);
    if (cost < best_cost - 1e-12) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

// Ring cell r of a TI x TJ tile -> tile coordinates (ii, jj), ii or jj just
// outside the tile (cross-shaped one-cell halo, no corners).
HF_HD inline void lns_ring_cell(const LeanTile& T, int r, int* ii, int* jj) {
  if (r < T.TJ) {
    *ii = -1;
    *jj = r;
  } else if (r < 2 * T.TJ) {
    *ii = T.TI;
    *jj = r - T.TJ;
  } else if (r < 2 * T.TJ + T.TI) {
    *ii = r - 2 * T.TJ;
    *jj = -1;
  } else {
    *ii = r - 2 * T.TJ - T.TI;
    *jj = T.TJ;
  }
}

// F_m of global cell (gi, gj) into LDS cell cc (committed S, A, B of the
// live equations); *early / *filled as fill_compute's.
template <int MODE, int TURB = 2>
HF_HD inline void lns_fill_to_lds(const StepParams& P, const LnsArrays& a, int gi, int gj, real* lds, int NC, int cc,
                                  CellLocal& c, bool* early, bool* filled, int* neg_dummy) {
  constexpr int NL = Lns<MODE>::NL;
  LnsFillIO<MODE, TURB> io(a, gi, gj, P.nx, P.ny);
  real mY[1], mgx[1], mgy[1];
  (void)fill_compute<MODE, 1, LnsFillIO<MODE, TURB>, true>(P, io, c, mY, mgx, mgy, nullptr, 0, gi, gj, true,
                                                             neg_dummy, early, filled);
#pragma unroll
  for (int q = 0; q < NL; q++) {
    const int k = Lns<MODE>::eqk(q);
    lds[q * NC + cc] = c.S[k];
    lds[(NL + q) * NC + cc] = (*early || !*filled) ? 0.0 : c.A[k];
    lds[(2 * NL + q) * NC + cc] = (*early || !*filled) ? 0.0 : c.B[k];
  }
}

}  // namespace hf2d
