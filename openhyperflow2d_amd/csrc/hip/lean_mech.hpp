// Lean mechanism-mode N-S step (SK_MECH: finite-rate species, laminar or
// k-omega SST): the split predict + fill pair of the scramjet path replaced by
// one LDS-tiled kernel per step with every flux recomputed in the tile, plus
// the compacted kinetics and a state kernel over the reacting cells only.
//
// Split stepper, step m (stepkern.hpp; reference FillNode2D + TurbModRANS2D,
// hyper_flow_node.hpp:373-957, over the two sweeps of DEEPS2D_Run,
// deeps2d_core.cpp:853-1244):
//   predict_m   S^m, fluxes A/B/F^m of 6 + (ns - 1) equations -> Sp^{m+1}
//   kinetics    species of Sp^{m+1} at constant rho, e -> S^{m+1} species
//   fill_{m+1}  T^{m+1} by Newton on e(T), fluxes A/B/F^{m+1}, dt_{m+1}
// ~2.3 KB of HBM traffic per cell and step: the 15 equations' fluxes are
// written by the fill and read back by the predictor.
//
// Lean path, step m (hf2d_lnm_step + kinetics + hf2d_lnm_hot):
//   1. G_m: the flux part of fill_m for the tile's 16 x 16 cells and their
//      cross-shaped ring, from Sp^m / post-kinetics species and the STORED
//      thermodynamic state of level m (T, p, Cp, k) -- fill_node runs with
//      MechMixTile, whose state() loads what the Newton produced one step
//      earlier and whose heat_flux() writes the species fluxes into LDS.  The
//      flow / turbulence S, A, B and the species A, B go to LDS only;
//   2. predict_m of the tile's cells from LDS (flow, then species one by one)
//      -> Sp^{m+1};
//   3. E_{m+1}: skip tests, velocity recovery, wall conditions and the Newton
//      T of the NEW state (mech_state_node, the same pieces fill_node runs,
//      physics.hpp) -> state level m+1 and dt_{m+1}, for every cell the
//      kinetics leave alone; reacting cells (T^m >= Tchem) go to a list;
//   4. kinetics (chem_fast / hiprtc list kernels) in place on the list;
//   5. hf2d_lnm_hot: E_{m+1} of the listed cells after their kinetics.
// Every value is produced by the same expressions, in the same order, as the
// split kernels, so the two paths are bitwise equal (tests/test_gpu_mechanism.py);
// the device solver switches between them (lnm_materialize = the split fill).
//
// Persistent per-cell traffic: Sp (6) + species (ns), beta (6 + ns - 1),
// lagged U/V/T, transport mu/lam/mu_t, state T/p/Cp/k, turbulence sources:
// ~0.7 KB per cell-step.
#pragma once

#include "lean_ns.hpp"

namespace hf2d {

constexpr int LNM_NSB = 9;   // species block of the kernel (mechanisms up to 9 species)
constexpr int LNM_TILE = 16;  // tile edge (256 cells, one per thread; the ring is exactly one wavefront)

struct LnmArrays {
  long N = 0;
  const MechData* mech = nullptr;
  int nsp = 0, bath = 0;
  const real* Sp = nullptr;   // Sp^m (flow + turbulence equations, [k * N + idx])
  real* Sp_out = nullptr;     // Sp^{m+1}
  const real* Ys = nullptr;   // species of S^m (after the kinetics), [s * N + idx]
  real* Ys_out = nullptr;     // species of Sp^{m+1} (the kinetics then update them in place)
  real* beta = nullptr;       // in place
  real* betas = nullptr;
  const real *Ui = nullptr, *Vi = nullptr, *Ti = nullptr;   // level m-1 (gradients, velocity recovery)
  real *Uo = nullptr, *Vo = nullptr, *To = nullptr;         // level m
  const real *mui = nullptr, *lami = nullptr, *mu_ti = nullptr;
  real *muo = nullptr, *lamo = nullptr, *mu_to = nullptr;
  const real *Tsi = nullptr, *psi = nullptr, *CPsi = nullptr, *ksi = nullptr;   // state of level m
  real *Tso = nullptr, *pso = nullptr, *CPso = nullptr, *kso = nullptr;         // state of level m+1
  const real *l_min = nullptr, *y_plus = nullptr, *BGX = nullptr, *BGY = nullptr, *grad = nullptr;
  real* Src = nullptr;      // turbulence sources, in place
  real* SrcAdd = nullptr;   // wall sources, in place
  const real *gA = nullptr, *gB = nullptr, *gF = nullptr;   // turbulence fluxes of nodes without the model
  const real* dSdx_in = nullptr;
  const real* dSdy_in = nullptr;
  real* dSdx_out = nullptr;
  real* dSdy_out = nullptr;
  const real* dSdxs_in = nullptr;   // species Cauchy dS (nullptr: no node needs them)
  const real* dSdys_in = nullptr;
  real* dSdxs_out = nullptr;
  real* dSdys_out = nullptr;
  const u64* CT = nullptr;
  const u64* TT = nullptr;
  const uint8_t* nb = nullptr;
  const uint8_t* gf = nullptr;
  int* hot = nullptr;   // reacting cells of the step (kinetics list)
  unsigned* hot_n = nullptr;   // ... and their count (DevScalars::hot_cnt / hot_cnt2 of the slot)
  int part = 0;   // tiles of this launch: 0 all, 1 the strip's edge tile columns, 2 the others (comm overlap)
  unsigned long long* tr = nullptr;   // phase trace (HF2D_LNM_TRACE): 12 clocks per workgroup
  // xGMI mailboxes: the previous step's HALO_LNS list (lg) and the exchange
  // arguments (xg, device copies): the edge tiles copy that step's halo from
  // the mailbox into the ghost columns first (fx_ghost_prologue)
  const struct FusedX* xg = nullptr;
  const struct ColList* lg = nullptr;
};

// Tile of the lean mechanism step: TI columns x LNM_TILE rows, one cell per
// thread.  TI = 16: the 64 ring cells take a second fill on wavefront 0;
// TI = 12: 192 own + 56 ring cells, every thread one fill.
inline LeanTile lnm_tile(int ncols, int ny, int ti) {
  LeanTile T;
  T.TJ = LNM_TILE;
  T.TI = T.TIh = ti;
  T.CPT = 1;
  T.W = T.TJ + 2;
  T.NC = (T.TI + 2) * T.W;
  T.nbi = (ncols + T.TI - 1) / T.TI;
  T.nbj = (ny + T.TJ - 1) / T.TJ;
  return T;
}

// LDS planes of a TI x TJ tile.  Flow / turbulence equation q (Lns<SK_SGT>::q):
// S over the tile + cross ring, A over the tile + left/right ring, B over the
// tile + up/down ring; species t (transported index, bath skipped): A and B.
// 16 x 16 with 9 species: 80,064 B, two workgroups per CU.
struct LnmLayout {
  int TI, TJ, NC, NA, NB, nspt;
  int oS, oA, oB, osA, osB;
  HF_HD LnmLayout(int ti, int tj, int nspt_) : TI(ti), TJ(tj), nspt(nspt_) {
    NC = (TI + 2) * (TJ + 2);
    NA = (TI + 2) * TJ;
    NB = TI * (TJ + 2);
    oS = 0;
    oA = 6 * NC;
    oB = oA + 6 * NA;
    osA = oB + 6 * NB;
    osB = osA + nspt * NA;
  }
  HF_HD int total() const { return osB + nspt * NB; }
  HF_HD int s_at(int ii, int jj) const { return (ii + 1) * (TJ + 2) + jj + 1; }
  HF_HD int a_at(int ii, int jj) const { return (jj >= 0 && jj < TJ) ? (ii + 1) * TJ + jj : -1; }
  HF_HD int b_at(int ii, int jj) const { return (ii >= 0 && ii < TI) ? ii * (TJ + 2) + jj + 1 : -1; }
};

// Mixture closure of fill_node inside the tile: the state comes from the
// stored level (mech_state_node wrote it with MechMix::state's expressions);
// the heat flux forms the species gradients after it (as MechMixLazy) and
// writes the species fluxes into the LDS planes this cell feeds.  R is not
// read by fill_node after the state (dt lives in mech_state_node).
template <class IO>
struct MechMixTile {
  static constexpr bool MECH = true;
  const MechData* m;
  const IO* io;
  real* lds;
  int oA, oB, NA, NB, aoff, boff;
  real dx_1_n, dy_1_m, T, p, CP, k;
  int nsp, bath;
  bool grad_on, nx0, ny0;
  template <class Nd>
  HF_HD void state(Nd& n) const {
    n.Tg = T;
    n.CP = CP;
    n.k = k;
    n.p = p;
  }
  template <class Nd>
  HF_HD void heat_flux(const Nd& n, real& qx, real& qy) const {
    constexpr int NSB = LNM_NSB;
    real ys[NSB], yR[NSB], yL[NSB], yU[NSB], yD[NSB];
#pragma unroll
    for (int s = 0; s < NSB; s++) {
      const int sl = s < nsp ? s : nsp - 1;
      ys[s] = io->Ys(sl);
      yR[s] = io->Ysn(sl, ND_R);
      yL[s] = io->Ysn(sl, ND_L);
      yU[s] = io->Ysn(sl, ND_U);
      yD[s] = io->Ysn(sl, ND_D);
    }
#pragma unroll
    for (int s = 0; s < NSB; s++) {
      if (s >= m->ns) break;
      real gx = 0.0, gy = 0.0;
      if (grad_on && s < nsp) {
        if (!nx0) gx = (yR[s] - yL[s]) * dx_1_n;
        if (!ny0) gy = (yU[s] - yD[s]) * dy_1_m;
      }
      const real h = mech_h_species(*m, s, n.Tg);
      qx += n.Diff * h * gx;
      qy += n.Diff * h * gy;
      if (s < nsp && s != bath) {
        const int t = s < bath ? s : s - 1;
        real a = ys[s] * n.U, b = ys[s] * n.V;
        const real rx = n.Diff * gx, ry = n.Diff * gy;
        a -= rx;
        b -= ry;
        // (axisymmetric F_s = FT * (ys V) - ry = B_s: FT is exactly 1)
        if (aoff >= 0) lds[oA + t * NA + aoff] = a;
        if (boff >= 0) lds[oB + t * NB + boff] = b;
      }
    }
  }
};

// fill_compute() accessor of a tile / ring cell: every input the fill reads
// is loaded up front at clamped neighbour indices (one memory latency), the
// neighbour bits select them later (a missing neighbour resolves to the cell
// itself, as FillSoAIO).  Inputs fill_node rewrites before any use return +0.
// TURB: fill_node's turbulence-model set (0 none, 3 SST).
template <int TURB>
struct LnmFillIO {
  static constexpr int TILE_TURB = TURB;
  using Mix = MechMixTile<LnmFillIO<TURB>>;
  const LnmArrays& a;
  long N, idx, nsel[4];
  u64 ct, tt;
  uint8_t g, b;
  real s[6], u, v, t, mu_, lam_, mut_, lmin_, yp_, Ts, ps, CPs, ks;
  real rn[4], un[4], vn[4], tn[4], kn[4], en[4];
  int nbit[4];
  // LDS targets of this cell's species fluxes (MechMixTile)
  real* lds = nullptr;
  const LnmLayout* L = nullptr;
  int aoff = -1, boff = -1;
  HF_HD LnmFillIO(const LnmArrays& aa, int i, int j, int nx, int ny) : a(aa), N(aa.N), idx((long)i * ny + j) {
    const long nbi[4] = {i > 0 ? idx - ny : idx, i < nx - 1 ? idx + ny : idx, j < ny - 1 ? idx + 1 : idx,
                         j > 0 ? idx - 1 : idx};
    ct = a.CT[idx];
    tt = a.TT[idx];
    g = a.gf[idx];
    b = a.nb[idx];
#pragma unroll
    for (int q = 0; q < 6; q++) s[q] = a.Sp[Lns<SK_SGT>::eqk(q) * N + idx];
    u = a.Ui[idx];
    v = a.Vi[idx];
    t = a.Ti[idx];
    mu_ = a.mui[idx];
    lam_ = a.lami[idx];
    mut_ = a.mu_ti[idx];
    lmin_ = a.l_min[idx];
    yp_ = a.y_plus[idx];
    Ts = a.Tsi[idx];
    ps = a.psi[idx];
    CPs = a.CPsi[idx];
    ks = a.ksi[idx];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      rn[d] = a.Sp[nbi[d]];
      un[d] = a.Ui[nbi[d]];
      vn[d] = a.Vi[nbi[d]];
      tn[d] = a.Ti[nbi[d]];
      kn[d] = TURB ? a.Sp[(long)I_K * N + nbi[d]] : 0.0;
      en[d] = TURB ? a.Sp[(long)I_EPS * N + nbi[d]] : 0.0;
      nbit[d] = 0;
      nsel[d] = idx;
    }
  }
  HF_HD void set_nb(int i, int j, int ny, int n1, int n2, int n3, int n4) {
    nbit[ND_L] = n1;
    nbit[ND_R] = n2;
    nbit[ND_U] = n3;
    nbit[ND_D] = n4;
    nsel[ND_L] = (long)(i - n1) * ny + j;
    nsel[ND_R] = (long)(i + n2) * ny + j;
    nsel[ND_U] = idx + n3;
    nsel[ND_D] = idx - n4;
  }
  HF_HD Mix mixer(const real*, real dx_1_n, real dy_1_m, bool active, bool nx0, bool ny0) const {
    Mix mx;
    mx.m = a.mech;
    mx.io = this;
    mx.lds = lds;
    mx.oA = L->osA;
    mx.oB = L->osB;
    mx.NA = L->NA;
    mx.NB = L->NB;
    mx.aoff = aoff;
    mx.boff = boff;
    mx.dx_1_n = dx_1_n;
    mx.dy_1_m = dy_1_m;
    mx.T = Ts;
    mx.p = ps;
    mx.CP = CPs;
    mx.k = ks;
    mx.nsp = a.nsp;
    mx.bath = a.bath;
    mx.grad_on = active;
    mx.nx0 = nx0;
    mx.ny0 = ny0;
    return mx;
  }
  HF_HD bool model() const { return TURB == 3 && has_all(tt, TCT_k_omega_SST_Model); }
  HF_HD u64 CT() const { return ct; }
  HF_HD u64 TT() const { return tt; }
  HF_HD uint8_t gf() const { return g; }
  HF_HD uint8_t nb() const { return b; }
  HF_HD real S(int k) const { return s[Lns<SK_SGT>::q(k)]; }
  HF_HD real Sn(int k, int d) const {
    if (k == 0) return nbit[d] ? rn[d] : s[0];
    if (k == I_K) return nbit[d] ? kn[d] : s[4];
    if (k == I_EPS) return nbit[d] ? en[d] : s[5];
    return 0.0;
  }
  HF_HD real A(int k) const { return model() ? 0.0 : a.gA[k * N + idx]; }
  HF_HD real B(int k) const { return model() ? 0.0 : a.gB[k * N + idx]; }
  HF_HD real F(int k) const { return model() ? 0.0 : a.gF[k * N + idx]; }
  HF_HD real Src(int k) const { return a.Src[k * N + idx]; }
  HF_HD real SrcAdd(int k) const { return a.SrcAdd[k * N + idx]; }
  HF_HD real Uo() const { return u; }
  HF_HD real Vo() const { return v; }
  HF_HD real To() const { return t; }
  HF_HD real Uon(int d) const { return nbit[d] ? un[d] : u; }
  HF_HD real Von(int d) const { return nbit[d] ? vn[d] : v; }
  HF_HD real Ton(int d) const { return nbit[d] ? tn[d] : t; }
  HF_HD real p() const { return ps; }      // rewritten by the state before any use
  HF_HD real kk() const { return ks; }     // skip test (mech_state_node decided it on the lagged k)
  HF_HD real R() const { return 0.0; }     // not read by fill_node (state, SST)
  HF_HD real CP() const { return CPs; }    // SST's lam_t before the state is rewritten after it
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
  // stored gradients are read only by nodes that do not recompute them (NT_FC)
  HF_HD real grad(int gg) const { return is_active(ct) ? 0.0 : a.grad[gg * N + idx]; }
  HF_HD real Ys(int sp) const { return a.Ys[(long)sp * N + idx]; }
  HF_HD real Ysn(int sp, int d) const { return a.Ys[(long)sp * N + nsel[d]]; }
};

// The own cell's level-m values kept in registers from G_m to the predictor
// and E_{m+1}.
struct LnmLevel {
  real U, V, Tg, k, BGX, BGY;
  real SrcAdd[6], F[6], Src[6];
};

// predict_core() accessor of the flow / turbulence equations: committed S and
// fluxes from the LDS planes, F / Src / SrcAdd of the own cell from registers.
struct LnmPredictIO {
  static constexpr int NE = NEQ;
  static constexpr bool skip(int k) { return !sk_live(SK_MECH, k); }
  HF_HD static constexpr int eq(int k) { return k; }
  HF_HD static constexpr int q(int k) { return Lns<SK_SGT>::q(k); }
  const LnmArrays& a;
  const real* lds;
  const LnmLayout& L;
  const LnmLevel& lv;
  const real* bpre;
  long N, idx, iL, iR, iU, iD;
  int sC, sL, sR, sU, sD, aL, aR, bU, bD;
  uint8_t gf;
  real sn[NEQ];
  HF_HD real S(int k) const { return lds[L.oS + q(k) * L.NC + sC]; }
  HF_HD real SL(int k) const { return lds[L.oS + q(k) * L.NC + sL]; }
  HF_HD real SR(int k) const { return lds[L.oS + q(k) * L.NC + sR]; }
  HF_HD real SU(int k) const { return lds[L.oS + q(k) * L.NC + sU]; }
  HF_HD real SD(int k) const { return lds[L.oS + q(k) * L.NC + sD]; }
  HF_HD real AL(int k) const { return lds[L.oA + q(k) * L.NA + aL]; }
  HF_HD real AR(int k) const { return lds[L.oA + q(k) * L.NA + aR]; }
  HF_HD real BU(int k) const { return lds[L.oB + q(k) * L.NB + bU]; }
  HF_HD real BD(int k) const { return lds[L.oB + q(k) * L.NB + bD]; }
  HF_HD real dxL(int k) const { return a.dSdx_in[k * N + iL]; }
  HF_HD real dxR(int k) const { return a.dSdx_in[k * N + iR]; }
  HF_HD real dyU(int k) const { return a.dSdy_in[k * N + iU]; }
  HF_HD real dyD(int k) const { return a.dSdy_in[k * N + iD]; }
  HF_HD real beta(int k) const { return bpre[q(k)]; }
  HF_HD real F(int k) const { return lv.F[q(k)]; }
  // SoAPredictIO: turbulence sources always, flow sources never (lnm_ok)
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

// predict_core() accessor of species s (SpeciesPredictIO with the fluxes in
// the LDS planes and the species' own / neighbour values and blending factor
// loaded before the workgroup barrier: a load after a store of the previous
// species cannot be hoisted, so per-species loads were one memory latency
// each).  F_s of the axisymmetric predictor equals B_s (FT = 1).
struct LnmSpeciesIO {
  static constexpr int NE = 1;
  static constexpr bool skip(int) { return false; }
  HF_HD static constexpr int eq(int) { return I_YFU; }
  const LnmArrays& a;
  const real* lds;
  const LnmLayout& L;
  long N, idx, iL, iR, iU, iD, o;
  int t, aL, aR, bU, bD, bC;
  uint8_t gf;
  real ys, yl, yr, yu, yd, bt, srcadd_rho, rho_c, out;
  HF_HD real S(int) const { return ys; }
  HF_HD real SL(int) const { return yl; }
  HF_HD real SR(int) const { return yr; }
  HF_HD real SU(int) const { return yu; }
  HF_HD real SD(int) const { return yd; }
  HF_HD real AL(int) const { return lds[L.osA + t * L.NA + aL]; }
  HF_HD real AR(int) const { return lds[L.osA + t * L.NA + aR]; }
  HF_HD real BU(int) const { return lds[L.osB + t * L.NB + bU]; }
  HF_HD real BD(int) const { return lds[L.osB + t * L.NB + bD]; }
  HF_HD real dxL(int) const { return a.dSdxs_in ? a.dSdxs_in[o + iL] : 0.0; }
  HF_HD real dxR(int) const { return a.dSdxs_in ? a.dSdxs_in[o + iR] : 0.0; }
  HF_HD real dyU(int) const { return a.dSdys_in ? a.dSdys_in[o + iU] : 0.0; }
  HF_HD real dyD(int) const { return a.dSdys_in ? a.dSdys_in[o + iD] : 0.0; }
  HF_HD real beta(int) const { return bt; }
  HF_HD real F(int) const { return lds[L.osB + t * L.NB + bC]; }
  HF_HD real Src(int) const { return 0.0; }
  HF_HD real SrcAdd(int) const { return (gf & GF_SRCADD) ? srcadd_rho * (ys / rho_c) : 0.0; }
  HF_HD void put_S(int, real v) {
    out = v;
    a.Ys_out[o + idx] = v;
  }
  HF_HD void put_beta(int, real v) const { a.betas[o + idx] = v; }
  HF_HD void put_dS(int, real x, real y) const {
    if ((gf & GF_DX_OUT) && a.dSdxs_out) a.dSdxs_out[o + idx] = x;
    if ((gf & GF_DY_OUT) && a.dSdys_out) a.dSdys_out[o + idx] = y;
  }
  HF_HD void keep_dS(int) const {
    if ((gf & GF_DX_OUT) && a.dSdxs_out) a.dSdxs_out[o + idx] = a.dSdxs_in[o + idx];
    if ((gf & GF_DY_OUT) && a.dSdys_out) a.dSdys_out[o + idx] = a.dSdys_in[o + idx];
  }
};

// E: the thermodynamic state of a set, non-solid node from its conserved
// flow state and species -- fill_compute's inputs and fill_node's
// fill_node_pre, fill_node_wall and MechMix::state in their order (the
// turbulence model between them touches none of these values) -- and, for an
// active node, the local dt and the T check of fill_compute.  False: fill_node
// would skip the node (rho = 0 or k < 1; the lean path cannot recompute the
// fluxes of a skipped node and stops).
struct LnmState {
  real T, p, CP, k;
};
HF_HD inline bool mech_state_node(const StepParams& P, const MechData& m, int nsp, const real* S4, const real* ys,
                                  real Ul, real Vl, real Tl, real kl, u64 CT, real bgx, real bgy, LnmState* st,
                                  real* dt_local, int* neg) {
  CellLocal c;
#pragma unroll
  for (int k = 0; k < NEQ; k++) {
    c.S[k] = k < 4 ? S4[k] : 0.0;
    c.SrcAdd[k] = 0.0;
  }
#pragma unroll
  for (int s = 0; s < NSPEC; s++) c.Y[s] = 0.0;
  c.CT = CT;
  c.U = Ul;
  c.V = Vl;
  c.Tg = Tl;
  c.k = kl;
  c.R = c.CP = c.p = 0.0;
  c.BGX = bgx;
  c.BGY = bgy;
  c.Uw = c.Vw = 0.0;
  real mY[LNM_NSB];
  const real rho = S4[I_RHO];
#pragma unroll
  for (int s = 0; s < LNM_NSB; s++) mY[s] = (s < nsp && rho != 0) ? ys[s] / rho : 0.0;
  *dt_local = 1.0;
  if (!fill_node_pre(c)) return false;
  fill_node_wall(c, P.fpa);
  MechMix<LNM_NSB>{&m, mY, nullptr, nullptr}.state(c);
  st->T = c.Tg;
  st->p = c.p;
  st->CP = c.CP;
  st->k = c.k;
  if (is_active(CT)) {
    if (c.Tg < 0. || !(c.Tg > MECH_TMIN)) {
      *neg = 1;
    } else {
      const real AAA = std::sqrt(c.k * c.R * c.Tg);
      *dt_local = P.CFL_min * hf_min(P.dx / (AAA + std::fabs(c.U)), P.dy / (AAA + std::fabs(c.V)));
    }
  }
  return true;
}

}  // namespace hf2d
