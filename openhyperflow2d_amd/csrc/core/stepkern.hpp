// Per-cell DEEPS step kernels over structure-of-arrays state, shared verbatim
// by the CPU Jacobi stepper and the HIP kernels (hip/kernels.hip), so the two
// agree to rounding.
//
// Jacobi semantics (the reference sweeps in place, Gauss-Seidel-like;
// SURVEY H1): every phase reads only values produced by the previous phase.
//   predict_cell   pass 1 + pass 2a of DEEPS2D_Run (deeps2d_core.cpp:853-1165):
//                  blended LxF/central predictor, BC handling, residual,
//                  blending-factor update, commit.  Reads S_in/A/B/F/dS*_in,
//                  writes S_out/dS*_out/beta.
//   fill_cell      pass 2b+2c (deeps2d_core.cpp:1169-1332): gradients from the
//                  committed neighbours (primitives U,V,T lagged one step),
//                  FillNode2D, negative-T check, local dt, chemistry.
//   wall_heat_*    CalcHeatOnWallSources (deeps2d_core.cpp:2679-2833) in
//                  owner-computes form (no scatter races).
#pragma once

#include <type_traits>

#include "physics.hpp"
#include "mechanism.hpp"
#include "mechanism_io.hpp"
#include "residual.hpp"

namespace hf2d {

// Neighbour-present bits packed per cell.
enum : uint8_t { NB_XL = 1, NB_XR = 2, NB_YU = 4, NB_YD = 8 };

// Per-cell traffic flags of the generic stepper (compute_generic_flags):
//   GF_DX_OUT / GF_DY_OUT  dS/dx, dS/dy of this node are read by a Cauchy
//                          (d2/dx2 = 0) neighbour, so they must be published
//   GF_SRC                 Src of the flow/species equations may be non-zero
//                          (sources, finite-rate chemistry)
//   GF_SRCADD              SrcAdd may be non-zero (wall nodes)
// Skipped loads are replaced by the +0 the arrays provably hold, skipped
// stores would rewrite unchanged values, so results are bit-identical.
//   GF_WBX / GF_WBY        Config::WallBlendCells: within that many cells of an
//                          x- / y-normal no-slip wall (predict_core drops the
//                          wall-normal neighbours from the tangential
//                          momentum's blend; read only with StepParams::wall_blend)
enum : uint8_t { GF_DX_OUT = 1, GF_DY_OUT = 2, GF_SRC = 4, GF_SRCADD = 8, GF_WBX = 16, GF_WBY = 32 };

// Raw SoA view.  Equation arrays are [k * N + idx], idx = i * ny + j
// (x-major, matching the .hf2d file; a column is contiguous).
struct SoA {
  int nx = 0, ny = 0;
  long N = 0;
  // conserved state and fluxes (equation-major)
  real* S = nullptr;
  real* A = nullptr;
  real* B = nullptr;
  real* F = nullptr;
  real* Src = nullptr;
  real* SrcAdd = nullptr;
  real* beta = nullptr;
  real* dSdx = nullptr;
  real* dSdy = nullptr;
  // primitives / transport
  real* U = nullptr;
  real* V = nullptr;
  real* Tg = nullptr;
  real* p = nullptr;
  real* kk = nullptr;   // Cp/Cv
  real* R = nullptr;
  real* CP = nullptr;
  real* lam = nullptr;
  real* mu = nullptr;
  real* mu_t = nullptr;
  real* lam_t = nullptr;
  real* Diff = nullptr;
  real* Y = nullptr;    // [NSPEC * N]
  // turbulence / wall data
  real* l_min = nullptr;
  real* y_plus = nullptr;
  real* Re_local = nullptr;
  real* BGX = nullptr;
  real* BGY = nullptr;
  real* Tf = nullptr;
  real* Q_conv = nullptr;
  real* grad = nullptr; // [10 * N]: dUdx dUdy dVdx dVdy dTdx dTdy dkdx dkdy depsdx depsdy
  u64* CT = nullptr;
  u64* TT = nullptr;
  uint8_t* nb = nullptr;
  uint8_t* gf = nullptr;   // GF_* flags (nullptr: all set)
  int32_t* wslot = nullptr;   // nearest wall of the cell: index into Case::wall_nodes (-1 none)
  // mechanism mode (SK_MECH): species partial densities and their fluxes,
  // blending factors and Cauchy dS, species-major [s * N + idx]
  const MechData* mech = nullptr;
  int nsp = 0;
  real* Ys = nullptr;
  real* As = nullptr;
  real* Bs = nullptr;
  real* Fs = nullptr;
  real* betas = nullptr;
  real* dSdxs = nullptr;   // nullptr unless some node applies d2(rhoY)/dx2 = 0
  real* dSdys = nullptr;
};

enum { G_DUDX = 0, G_DUDY, G_DVDX, G_DVDY, G_DTDX, G_DTDY, G_DKDX, G_DKDY, G_DEDX, G_DEDY, NGRAD };

// CFL / blending-factor scenario tables (deck CFL_Scenario, beta_Scenario)
// for device-side evaluation: the device kernels read the iteration number
// from device memory, so a captured step graph stays valid while the
// scenario ramps.
struct ScenarioTables {
  TableData cfl, beta;
  real CFL = 0, beta0 = 0;
};

struct StepParams {
  int nx, ny;        // local array extents (including halo columns)
  int i0, i1;        // owned/computed column range [i0, i1)
  int gx0;           // global column index of local column 0
  real dx, dy, dt;
  real dtdx, dtdy, dxx, dyy;  // dxx = dy/(dx+dy), dyy = dx/(dx+dy)
  real beta_min;     // min(beta0, beta_Scenario(it))
  real nrbc_beta0;
  real CFL_min;      // min(CFL, CFL_Scenario(it))
  real visc_cfl;     // Config::ViscousCFL (0: inviscid CFL only, as the reference)
  int bff;
  int alternate_rms;
  int do_residual;
  int sm;            // ProblemType
  int chem_model;
  FillParams fpa;    // for active cells (is_mu_t / is_init per TurbStartIter)
  FillParams ffc;    // for NT_FC cells: FillNode2D(1, 0, ...)
  const SpeciesProps* species;  // host or device pointer
  const ScenarioTables* scen = nullptr;   // device: evaluate beta_min / CFL_min per step
  int xcd = 0;       // device split kernels: XCD-aware workgroup order (speed only; host ignores it)
  // device tile kernels: workgroup w waits (w / stagger_wgs) * stagger ticks
  // of the 100 MHz clock before staging, so the dispatch rounds of a
  // co-resident grid load their tiles one after another (speed only)
  int stagger = 0, stagger_wgs = 256;
  // Config::LaggedDt: the step's dt is the all-rank MIN of two steps back
  // (device: DevScalars::dt_lag; host: SolverBase::dt_lag)
  int lag_dt = 0;
  int wall_blend = 0;   // Config::WallBlendCells > 0: predictor accessors' gf carries GF_WBX / GF_WBY
  real wall_blend_f = 0;   // Config::WallBlendFactor
  // device solver, single GPU: the last step of a host call publishes its
  // scalars (dt, error flag, time) into the pinned host mirror itself
  // (hip/device_solver.hip host_tail; nullptr: hf2d_scalars_out does it)
  void* host_sc = nullptr;
  unsigned* host_done = nullptr;
  // device lean tile kernel, single GPU (speed only, the value is the same):
  // dt_fold = 1: the last workgroup to finish folds the dt shards of the next
  // slot into its word (completion count on host_done); dt_read = 2: the
  // step reads only the word (the previous launch folded), 1: the word and
  // the shards with one vector load per lane, 0: with scalar loads
  int dt_fold = 0, dt_read = 0;
  // lean tile kernel: stores of the in-place per-cell arrays (beta, CP) are
  // skipped when the new value has the old value's bits (converged regions;
  // speed only -- the array holds the same bits either way)
  int skip_same = 0;
};

// Register-resident cell used by fill_node / turb_model / chemistry.
struct CellLocal {
  real S[NEQ], A[NEQ], B[NEQ], F[NEQ], RX[NEQ], RY[NEQ], Src[NEQ], SrcAdd[NEQ];
  real U, V, p, Tg, k, R, CP, lam, mu, Diff, mu_t, lam_t;
  real l_min, y_plus, Re_local;
  real dkdx, dkdy, depsdx, depsdy;
  real dUdx, dUdy, dVdx, dVdy, dTdx, dTdy;
  real droYdx[NSPEC], droYdy[NSPEC];
  real Y[NSPEC];
  real BGX, BGY, Uw, Vw, y, Tf;
  u64 CT, TurbType;
};

// ---------------------------------------------------------------------------
// Equation BC masks (deeps2d_core.cpp:903-991).  Returns false when the
// equation is frozen (Dirichlet or not transported for this cell model).
// ---------------------------------------------------------------------------
struct EqFlags {
  bool upd;   // not Dirichlet
  bool dx, dy, dx2, dy2;   // dx/dy: flux difference used (no Neumann); dx2/dy2: Cauchy
};

HF_HD inline EqFlags eq_flags(int k, u64 CT, u64 TT, int sm) {
  EqFlags f{false, true, true, false, false};
  if (k < 4) {
    f.upd = !has_all(CT, CT_Rho_CONST << k);
    f.dx = !has_all(CT, CT_dRhodx_NULL << k);
    f.dy = !has_all(CT, CT_dRhody_NULL << k);
    f.dx2 = has_all(CT, CT_d2Rhodx2_NULL << k);
    f.dy2 = has_all(CT, CT_d2Rhody2_NULL << k);
  } else if (k < 4 + NCOMP) {
    f.upd = !has_all(CT, CT_Y_CONST);
    f.dx = !has_all(CT, CT_dYdx_NULL);
    f.dy = !has_all(CT, CT_dYdy_NULL);
    f.dx2 = has_all(CT, CT_d2Ydx2_NULL);
    f.dy2 = has_all(CT, CT_d2Ydy2_NULL);
  } else if (sm == SM_NS && has_turb_eq(TT)) {
    // The reference shifts the eps masks by (k - 7) as well, so eps tests
    // the *next* flag bit (quirk Q3, kept for parity).
    const int sh = k - 4 - NCOMP;
    const bool e = (k == I_EPS);
    f.upd = !has_all(TT, (e ? TCT_eps_CONST : TCT_k_CONST) << sh);
    f.dx = !has_all(TT, (e ? TCT_depsdx_NULL : TCT_dkdx_NULL) << sh);
    f.dy = !has_all(TT, (e ? TCT_depsdy_NULL : TCT_dkdy_NULL) << sh);
    f.dx2 = has_all(TT, (e ? TCT_d2epsdx2_NULL : TCT_d2kdx2_NULL) << sh);
    f.dy2 = has_all(TT, (e ? TCT_d2epsdy2_NULL : TCT_d2kdy2_NULL) << sh);
  }
  return f;
}

// Pass-2 "Dirichlet" test used to gate the residual/beta update: for the
// turbulence equations the reference tests TCT bits against CT (quirk Q4).
HF_HD inline bool pass2_frozen(int k, u64 CT, u64 TT, int sm) {
  u64 c = 0;
  if (k < 4)
    c = CT_Rho_CONST << k;
  else if (k < 4 + NCOMP)
    c = CT_Y_CONST;
  else if (sm == SM_NS && has_turb_eq(TT))
    c = TCT_k_CONST << (k - 4 - NCOMP);
  return has_all(CT, c);
}

HF_HD inline bool is_active(u64 CT) {
  return has_all(CT, CT_NODE_IS_SET) && !has_all(CT, CT_SOLID) && !has_all(CT, NT_FC);
}

HF_HD inline real blend_beta(int bff, real beta_min, real beta_old, real DD, real sqrt_res) {
  const real b2 = beta_min * beta_min;
  switch (bff) {
    case BFF_L: return hf_min(beta_min, hf_div(b2, beta_min + DD));
    case BFF_LR: return hf_min((beta_min + beta_old) * 0.5, hf_div(b2, beta_min + DD));
    case BFF_S: return hf_min(beta_min, hf_div(b2, beta_min + DD * DD));
    case BFF_SR: return hf_min((beta_min + beta_old) * 0.5, hf_div(b2, beta_min + DD * DD));
    case BFF_SQR: return hf_min(beta_min, hf_div(b2, beta_min + sqrt_res));
    case BFF_SQRR: return hf_min((beta_min + beta_old) * 0.5, hf_div(b2, beta_min + sqrt_res));
    default: return beta_old;   // declared but unimplemented variants (Q22)
  }
}

// ---------------------------------------------------------------------------
// Pass 1 + pass 2a for one active cell, written once against an accessor so
// the generic SoA stepper and the lean Euler kernel (fluxes recomputed from
// the neighbours' state instead of loaded) share the exact arithmetic.
//
// IO must provide (k = equation; L/R/U/D are the neighbour slots iL/iR/iU/iD,
// which resolve to the cell itself when the neighbour is absent):
//   S(k)  SL(k) SR(k) SU(k) SD(k)      conserved state
//   AL(k) AR(k) BU(k) BD(k)            fluxes at the neighbour slots
//   dxL(k) dxR(k) dyU(k) dyD(k)        previous dS/dx, dS/dy (Cauchy BCs)
//   beta(k) F(k) Src(k) SrcAdd(k)
//   put_S(k, v) put_beta(k, v) put_dS(k, dsdx, dsdy) keep_dS(k)
// ---------------------------------------------------------------------------
//
// PLAIN: the caller guarantees an interior node whose IO::NE equations are
// all transported with plain flux differences (no Dirichlet / Neumann /
// Cauchy bit, not frozen in pass 2, all four neighbours present, not
// non-reflecting).  The flags then fold to constants; the arithmetic is the
// same, so the result is bit-identical to the general path.
// predictor accessors that carry the Config::WallBlendCells flags (a static
// member kWallBlend): only the split path's SoAPredictIO, so the lean N-S /
// mechanism tile kernels compile the blend out (the device solver sends a
// WallBlendCells deck down the split path)
template <class IO, class = void>
struct io_wall_blend : std::false_type {};
template <class IO>
struct io_wall_blend<IO, std::void_t<decltype(IO::kWallBlend)>> : std::bool_constant<IO::kWallBlend> {};

template <bool RES, class IO, bool PLAIN = false>
HF_HD inline void predict_core(const StepParams& P, IO& io, u64 CT, u64 TT, int n1, int n2, int n3, int n4, int gi,
                               int j, ResidualPack& rp) {
  // RES is a template flag (not a nullable pointer) so the device kernels
  // keep the residual pack in registers.
  if (PLAIN) n1 = n2 = n3 = n4 = 1;
  // 1 / max(n1 + n2, 1) with n in {0, 1}: exactly 0.5 or 1 (no division)
  const real n_n_1 = (n1 + n2 > 1) ? 0.5 : 1.0;
  const real m_m_1 = (n3 + n4 > 1) ? 0.5 : 1.0;
  const int Num_Eq = PLAIN ? NEQ : num_eq_for(TT);
  const bool axi = P.fpa.FT != 0;
#pragma unroll
  for (int kk = 0; kk < IO::NE; kk++) {
    if (IO::skip(kk)) continue;   // equation not stored by this accessor (single-gas species)
    // k: the reference equation whose BC masks / residual slot apply (the
    // mechanism species accessor maps every species to the species group)
    const int k = io.eq(kk);
    real s = io.S(kk);
    const EqFlags f = PLAIN ? EqFlags{true, true, true, false, false} : eq_flags(k, CT, TT, P.sm);
    if (!PLAIN &&
        (k >= Num_Eq || !f.upd || (k >= 4 + NCOMP && !(P.sm == SM_NS && has_turb_eq(TT))))) {
      // A TCT-frozen turbulence equation whose CT-based pass-2 test says
      // "not frozen" (quirk Q4) is scored against the never-written
      // predictor scratch (0) in the reference: DD = 1, dS = -S.
      if (k < Num_Eq && !f.upd && k >= 4 + NCOMP && P.sm == SM_NS && has_turb_eq(TT) &&
          !pass2_frozen(k, CT, TT, P.sm) && s != 0.) {
        const real beta = io.beta(kk);
        const real DD = 1.0;
        const real bmin = has_all(CT, CT_NONREFLECTED) ? P.nrbc_beta0 : P.beta_min;
        io.put_beta(kk, blend_beta(P.bff, bmin, beta, DD, 1.0));
        if (RES) {
          EqResidual& e = rp.eq[k];
          if (DD >= e.dd_max) {
            e.dd_max = DD;
            e.i = gi;
            e.j = j;
          }
          if (P.alternate_rms) {
            e.rms += s * s;
            e.sum_div += s * s;
          } else {
            e.rms += DD * DD;
            e.count += 1;
          }
        }
      }
      io.put_S(kk, s);
      io.keep_dS(kk);
      continue;
    }
    real dXX, dYY, dsdx, dsdy;
    if (f.dx) {
      dXX = dsdx = (io.AR(kk) - io.AL(kk)) * n_n_1;
    } else {
      // a missing neighbour resolves to the cell itself
      const real sL = n1 ? io.SL(kk) : s, sR = n2 ? io.SR(kk) : s;
      s = (sL * n2 + sR * n1) * n_n_1;
      dXX = dsdx = 0.;
    }
    if (f.dy) {
      dYY = dsdy = (io.BU(kk) - io.BD(kk)) * m_m_1;
    } else {
      const real sU = n3 ? io.SU(kk) : s, sD = n4 ? io.SD(kk) : s;
      s = (sU * n3 + sD * n4) * m_m_1;
      dYY = dsdy = 0.;
    }
    if (f.dx2) dXX = (io.dxL(kk) + io.dxR(kk)) * 0.5;
    if (f.dy2) dYY = (io.dyU(kk) + io.dyD(kk)) * 0.5;
    real SL = n1 ? io.SL(kk) : s, SR = n2 ? io.SR(kk) : s;
    real SU = n3 ? io.SU(kk) : s, SD = n4 ? io.SD(kk) : s;
    if constexpr (io_wall_blend<IO>::value) {
      // Config::WallBlendCells: the tangential momentum's blend leaves out
      // the wall-normal neighbours near a no-slip wall
      if (!PLAIN && __builtin_expect(P.wall_blend != 0, 0)) {
        const real f = P.wall_blend_f;
        if (k == I_RHOU && (io.gf & GF_WBY)) {
          SU = s + f * (SU - s);
          SD = s + f * (SD - s);
        }
        if (k == I_RHOV && (io.gf & GF_WBX)) {
          SL = s + f * (SL - s);
          SR = s + f * (SR - s);
        }
      }
    }
    const real beta = io.beta(kk);
    const real _beta = 1. - beta;
    real snew;
    if (axi)
      snew = s * beta + _beta * (P.dxx * (SL + SR) + P.dyy * (SU + SD)) * 0.5 -
             (P.dtdx * dXX + P.dtdy * (dYY + io.F(kk) / (j + 1))) + (io.Src(kk)) * P.dt + io.SrcAdd(kk);
    else
      snew = s * beta + _beta * (P.dxx * (SL + SR) + P.dyy * (SU + SD)) * 0.5 - (P.dtdx * dXX + P.dtdy * dYY) +
             (io.Src(kk)) * P.dt + io.SrcAdd(kk);
    io.put_dS(kk, dsdx, dsdy);
    // pass 2a: residual + blending factor
    if ((PLAIN || !pass2_frozen(k, CT, TT, P.sm)) && s != 0.) {
      const real absDD = snew - s;
      real DD, sqrt_res = 0;
      if (std::fabs(s) > 1.e-15) {
        DD = std::fabs(hf_div(absDD, s));
        // only the square-root blending variants read it (uniform branch)
        if (P.bff == BFF_SQR || P.bff == BFF_SQRR) sqrt_res = hf_sqrt(DD);
      } else {
        DD = 1.0;
      }
      const real bmin = (!PLAIN && has_all(CT, CT_NONREFLECTED)) ? P.nrbc_beta0 : P.beta_min;
      io.put_beta(kk, blend_beta(P.bff, bmin, beta, DD, sqrt_res));
      if (RES) {
        EqResidual& e = rp.eq[k];
        if (DD >= e.dd_max) {
          e.dd_max = DD;
          e.i = gi;
          e.j = j;
        }
        if (P.alternate_rms) {
          e.rms += absDD * absDD;
          e.sum_div += s * s;
        } else {
          e.rms += DD * DD;
          e.count += 1;
        }
      }
    }
    io.put_S(kk, snew);
  }
}

// Specialisations of the generic (split) stepper, selected on the host:
//   SK_GENERIC  every field of the reference record
//   SK_SGL      single-gas laminar N-S: equations 0..3 only
//   SK_SGT      single-gas N-S with a turbulence model: equations 0..3, 7, 8
// Species partial densities are +0 and stay so in both specialisations (the
// argument of the lean single-gas path), so their equations, fluxes, mixture
// fractions and R need not move through memory (sk_eligible on the host).
//   SK_MECH     mechanism mode: equations 0..3, 7, 8 of the record (its species
//               slots are 0) + the mechanism species block (SoA::Ys)
enum { SK_GENERIC = 0, SK_SGL = 1, SK_SGT = 2, SK_MECH = 3 };
HF_HD constexpr bool sk_live(int mode, int k) {
  return mode == SK_GENERIC || k < 4 || ((mode == SK_SGT || mode == SK_MECH) && k >= 4 + NCOMP);
}

// Accessor over the full SoA arrays (fluxes loaded).
template <int MODE = SK_GENERIC>
struct SoAPredictIO {
  static constexpr int NE = MODE == SK_SGL ? 4 : NEQ;
  static constexpr bool kWallBlend = true;
  static constexpr bool skip(int k) { return !sk_live(MODE, k); }
  HF_HD static constexpr int eq(int k) { return k; }
  const SoA& in;
  const SoA& out;
  long N, idx, iL, iR, iU, iD;
  HF_HD real S(int k) const { return in.S[k * N + idx]; }
  HF_HD real SL(int k) const { return in.S[k * N + iL]; }
  HF_HD real SR(int k) const { return in.S[k * N + iR]; }
  HF_HD real SU(int k) const { return in.S[k * N + iU]; }
  HF_HD real SD(int k) const { return in.S[k * N + iD]; }
  HF_HD real AL(int k) const { return in.A[k * N + iL]; }
  HF_HD real AR(int k) const { return in.A[k * N + iR]; }
  HF_HD real BU(int k) const { return in.B[k * N + iU]; }
  HF_HD real BD(int k) const { return in.B[k * N + iD]; }
  HF_HD real dxL(int k) const { return in.dSdx[k * N + iL]; }
  HF_HD real dxR(int k) const { return in.dSdx[k * N + iR]; }
  HF_HD real dyU(int k) const { return in.dSdy[k * N + iU]; }
  HF_HD real dyD(int k) const { return in.dSdy[k * N + iD]; }
  HF_HD real beta(int k) const { return in.beta[k * N + idx]; }
  HF_HD real F(int k) const { return in.F[k * N + idx]; }
  HF_HD real Src(int k) const { return (k >= 4 + NCOMP || (gf & GF_SRC)) ? in.Src[k * N + idx] : 0.0; }
  HF_HD real SrcAdd(int k) const { return (gf & GF_SRCADD) ? in.SrcAdd[k * N + idx] : 0.0; }
  HF_HD void put_S(int k, real v) const { out.S[k * N + idx] = v; }
  HF_HD void put_beta(int k, real v) const { out.beta[k * N + idx] = v; }
  HF_HD void put_dS(int k, real a, real b) const {
    if (gf & GF_DX_OUT) out.dSdx[k * N + idx] = a;
    if (gf & GF_DY_OUT) out.dSdy[k * N + idx] = b;
  }
  HF_HD void keep_dS(int k) const {
    if (gf & GF_DX_OUT) out.dSdx[k * N + idx] = in.dSdx[k * N + idx];
    if (gf & GF_DY_OUT) out.dSdy[k * N + idx] = in.dSdy[k * N + idx];
  }
  uint8_t gf = 0xff;
};

// Accessor over one species s of the mechanism block (SK_MECH): the
// reference's species-group BC masks and residual slot (I_YFU); no volume
// source (the kinetics are operator-split), the no-slip wall source of the
// species is SrcAdd_rho * Y_s like the reference's slots
// (hyper_flow_node.hpp FillNode2D, SrcAdd[4+i] = SrcAdd[0] * Y[i]).
struct SpeciesPredictIO {
  static constexpr int NE = 1;
  static constexpr bool skip(int) { return false; }
  HF_HD static constexpr int eq(int) { return I_YFU; }
  const SoA& in;
  const SoA& out;
  long N, idx, iL, iR, iU, iD;
  uint8_t gf;
  long o;   // s * N
  HF_HD real S(int) const { return in.Ys[o + idx]; }
  HF_HD real SL(int) const { return in.Ys[o + iL]; }
  HF_HD real SR(int) const { return in.Ys[o + iR]; }
  HF_HD real SU(int) const { return in.Ys[o + iU]; }
  HF_HD real SD(int) const { return in.Ys[o + iD]; }
  HF_HD real AL(int) const { return in.As[o + iL]; }
  HF_HD real AR(int) const { return in.As[o + iR]; }
  HF_HD real BU(int) const { return in.Bs[o + iU]; }
  HF_HD real BD(int) const { return in.Bs[o + iD]; }
  HF_HD real dxL(int) const { return in.dSdxs ? in.dSdxs[o + iL] : 0.0; }
  HF_HD real dxR(int) const { return in.dSdxs ? in.dSdxs[o + iR] : 0.0; }
  HF_HD real dyU(int) const { return in.dSdys ? in.dSdys[o + iU] : 0.0; }
  HF_HD real dyD(int) const { return in.dSdys ? in.dSdys[o + iD] : 0.0; }
  HF_HD real beta(int) const { return in.betas[o + idx]; }
  HF_HD real F(int) const { return in.Fs[o + idx]; }
  HF_HD real Src(int) const { return 0.0; }
  HF_HD real SrcAdd(int) const {
    return (gf & GF_SRCADD) ? in.SrcAdd[(long)I_RHO * N + idx] * (in.Ys[o + idx] / in.S[idx]) : 0.0;
  }
  HF_HD void put_S(int, real v) const { out.Ys[o + idx] = v; }
  HF_HD void put_beta(int, real v) const { out.betas[o + idx] = v; }
  HF_HD void put_dS(int, real a, real b) const {
    if ((gf & GF_DX_OUT) && out.dSdxs) out.dSdxs[o + idx] = a;
    if ((gf & GF_DY_OUT) && out.dSdys) out.dSdys[o + idx] = b;
  }
  HF_HD void keep_dS(int) const {
    if ((gf & GF_DX_OUT) && out.dSdxs) out.dSdxs[o + idx] = in.dSdxs[o + idx];
    if ((gf & GF_DY_OUT) && out.dSdys) out.dSdys[o + idx] = in.dSdys[o + idx];
  }
};

template <bool RES, int MODE = SK_GENERIC>
HF_HD inline void predict_cell_t(const StepParams& P, const SoA& in, const SoA& out, int i, int j,
                                 ResidualPack& res) {
  const long N = in.N;
  const long idx = (long)i * P.ny + j;
  const u64 CT = in.CT[idx];
  const uint8_t gf = in.gf ? in.gf[idx] : (uint8_t)0xff;
  if (!is_active(CT)) {
    for (int k = 0; k < NEQ; k++) {
      if (!sk_live(MODE, k)) continue;
      out.S[k * N + idx] = in.S[k * N + idx];
      if (gf & GF_DX_OUT) out.dSdx[k * N + idx] = in.dSdx[k * N + idx];
      if (gf & GF_DY_OUT) out.dSdy[k * N + idx] = in.dSdy[k * N + idx];
    }
    if (MODE == SK_MECH)
      for (int s = 0; s < in.nsp; s++) {
        const long o = (long)s * N + idx;
        out.Ys[o] = in.Ys[o];
        if ((gf & GF_DX_OUT) && out.dSdxs) out.dSdxs[o] = in.dSdxs[o];
        if ((gf & GF_DY_OUT) && out.dSdys) out.dSdys[o] = in.dSdys[o];
      }
    return;
  }
  const u64 TT = in.TT[idx];
  const uint8_t nbm = in.nb[idx];
  const int n1 = (nbm & NB_XL) ? 1 : 0, n2 = (nbm & NB_XR) ? 1 : 0;
  const int n3 = (nbm & NB_YU) ? 1 : 0, n4 = (nbm & NB_YD) ? 1 : 0;
  const long iL = (long)(i - n1) * P.ny + j, iR = (long)(i + n2) * P.ny + j;
  SoAPredictIO<MODE> io{in, out, N, idx, iL, iR, idx + n3, idx - n4, gf};
  predict_core<RES>(P, io, CT, TT, n1, n2, n3, n4, P.gx0 + i, j, res);
  if (MODE == SK_MECH) {
    // transported species, then the bath gas as the remainder of the new rho
    const int bath = in.mech->bath;
    real sum = 0.0;
    for (int s = 0; s < in.nsp; s++) {
      if (s == bath) continue;
      SpeciesPredictIO sio{in, out, N, idx, iL, iR, idx + n3, idx - n4, gf, (long)s * N};
      predict_core<RES>(P, sio, CT, TT, n1, n2, n3, n4, P.gx0 + i, j, res);
      sum += out.Ys[(long)s * N + idx];
    }
    out.Ys[(long)bath * N + idx] = out.S[idx] - sum;
  }
}

HF_HD inline void predict_cell(const StepParams& P, const SoA& in, const SoA& out, int i, int j,
                               ResidualPack* res) {
  if (res) {
    predict_cell_t<true>(P, in, out, i, j, *res);
  } else {
    ResidualPack d;
    predict_cell_t<false>(P, in, out, i, j, d);
  }
}

// ---------------------------------------------------------------------------
// Gradients + FillNode2D + dt + chemistry for one cell.
// `sin` holds the committed state (S after predict), prim_old the previous
// step's U/V/Tg.  Non-double-buffered per-cell fields are read from `sin`
// and written to `out` (the same arrays except A/B in the fused Euler path).
// Returns the local dt (1.0 when the cell does not limit dt); sets *neg_T.
// ---------------------------------------------------------------------------
// MODE (SK_*, see SoAPredictIO): the specialisations load and store only the
// live equations and the fields the next step reads (S, A, B, F, Src, SrcAdd
// of live equations; U, V, Tg, p, k, CP, lam, mu; SGT also the turbulence
// fields); chemistry reduces to chemistry_single_gas_ns(); output-only fields
// (SGL: Diff, grad) are written when store_grad (the host reads the record
// after this step).  Every field equals the generic path (GPU tests).
// Mechanism-mode mixture closure of fill_node (physics.hpp RefMix): T from
// rho*E by Newton on the thermally perfect e(T) of the current composition,
// then R, Cp, k = Cp/Cv and p = rho R T at that T; the species enthalpy
// diffusion term uses the absolute species enthalpies h_s(T).
template <int NSB>
struct MechMix {
  static constexpr bool MECH = true;
  const MechData* m;
  const real* Y;    // mass fractions
  const real* gx;   // d(rho Y_s)/dx, d(rho Y_s)/dy
  const real* gy;
  template <class N>
  HF_HD void state(N& n) const {
    const real rho = n.S[I_RHO];
    const real e = hf_div(n.S[I_RHOE] - rho * (n.U * n.U + n.V * n.V) * 0.5, rho);
    const real T = mech_T_from_e<NSB>(*m, Y, e, n.Tg);
    real ee, cv, R, cp;
    mech_mix_thermo<NSB>(*m, Y, T, &ee, &cv, &R, &cp);
    n.Tg = T;
    n.R = R;
    n.CP = cp;
    n.k = hf_div(cp, cv);
    n.p = rho * R * T;
  }
  template <class N>
  HF_HD void heat_flux(const N& n, real& qx, real& qy) const {
#pragma unroll
    for (int s = 0; s < NSB; s++) {
      if (s >= m->ns) break;
      const real h = mech_h_species(*m, s, n.Tg);
      qx += n.Diff * h * gx[s];
      qy += n.Diff * h * gy[s];
    }
  }
};

// Input accessor of fill_compute() over the split stepper's SoA arrays:
// `sin` the committed state (and the per-cell fields of the last fill),
// `pold` the previous fill's primitives.  Neighbour reads go through the
// direction codes ND_* after set_nb() (a missing neighbour resolves to the
// cell itself).  The lean N-S kernel (lean_ns.hpp) supplies the same values
// from its own buffers / LDS, so both paths run the same arithmetic.
enum { ND_L = 0, ND_R, ND_U, ND_D };
struct FillSoAIO {
  const SoA& sin;
  const SoA& pold;
  long N, idx, nbi[4];
  HF_HD FillSoAIO(const SoA& s, const SoA& po, long i) : sin(s), pold(po), N(s.N), idx(i), nbi{i, i, i, i} {}
  HF_HD void set_nb(int i, int j, int ny, int n1, int n2, int n3, int n4) {
    nbi[ND_L] = (long)(i - n1) * ny + j;
    nbi[ND_R] = (long)(i + n2) * ny + j;
    nbi[ND_U] = idx + n3;
    nbi[ND_D] = idx - n4;
  }
  HF_HD u64 CT() const { return sin.CT[idx]; }
  HF_HD u64 TT() const { return sin.TT[idx]; }
  HF_HD uint8_t gf() const { return sin.gf ? sin.gf[idx] : (uint8_t)0xff; }
  HF_HD uint8_t nb() const { return sin.nb[idx]; }
  HF_HD bool inplace(const SoA& out) const { return sin.A == out.A && sin.B == out.B && sin.F == out.F; }
  HF_HD real S(int k) const { return sin.S[k * N + idx]; }
  HF_HD real Sn(int k, int d) const { return sin.S[k * N + nbi[d]]; }
  HF_HD real A(int k) const { return sin.A[k * N + idx]; }
  HF_HD real B(int k) const { return sin.B[k * N + idx]; }
  HF_HD real F(int k) const { return sin.F[k * N + idx]; }
  HF_HD real Src(int k) const { return sin.Src[k * N + idx]; }
  HF_HD real SrcAdd(int k) const { return sin.SrcAdd[k * N + idx]; }
  HF_HD real Uo() const { return pold.U[idx]; }
  HF_HD real Vo() const { return pold.V[idx]; }
  HF_HD real To() const { return pold.Tg[idx]; }
  HF_HD real Uon(int d) const { return pold.U[nbi[d]]; }
  HF_HD real Von(int d) const { return pold.V[nbi[d]]; }
  HF_HD real Ton(int d) const { return pold.Tg[nbi[d]]; }
  HF_HD real p() const { return sin.p[idx]; }
  HF_HD real kk() const { return sin.kk[idx]; }
  HF_HD real R() const { return sin.R[idx]; }
  HF_HD real CP() const { return sin.CP[idx]; }
  HF_HD real lam() const { return sin.lam[idx]; }
  HF_HD real mu() const { return sin.mu[idx]; }
  HF_HD real Diff() const { return sin.Diff[idx]; }
  HF_HD real mu_t() const { return sin.mu_t[idx]; }
  HF_HD real lam_t() const { return sin.lam_t[idx]; }
  HF_HD real l_min() const { return sin.l_min[idx]; }
  HF_HD real y_plus() const { return sin.y_plus[idx]; }
  HF_HD real Re_local() const { return sin.Re_local[idx]; }
  HF_HD real BGX() const { return sin.BGX[idx]; }
  HF_HD real BGY() const { return sin.BGY[idx]; }
  HF_HD real Tf() const { return sin.Tf[idx]; }
  HF_HD real Y(int s) const { return sin.Y[s * N + idx]; }
  HF_HD real grad(int g) const { return sin.grad[g * N + idx]; }
  HF_HD real Ys(int s) const { return sin.Ys[(long)s * N + idx]; }
  HF_HD real Ysn(int s, int d) const { return sin.Ys[(long)s * N + nbi[d]]; }
};

// MechMix whose species gradients are formed inside heat_flux() (after the
// Newton recovery of T) instead of before fill_node(), and which stores the
// species fluxes right there (the split mechanism fill, N-S): the gradient
// and flux registers are not live across the Newton iteration.  Same loads,
// same expressions, same order as fill_compute's gradient loop, MechMix's
// heat flux and fill_cell's species-flux loop: bitwise equal.
template <int NSB, class IO>
struct MechMixLazy {
  static constexpr bool MECH = true;
  const MechData* m;
  const real* Y;
  IO* io;
  const SoA* out;
  long N, idx;
  real dx_1_n, dy_1_m, FT;
  int nsp, bath;
  bool grad_on, nx0, ny0, axi;
  template <class Nd>
  HF_HD void state(Nd& n) const {
    MechMix<NSB>{m, Y, nullptr, nullptr}.state(n);
  }
  template <class Nd>
  HF_HD void heat_flux(const Nd& n, real& qx, real& qy) const {
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
        const long o = (long)s * N + idx;
        real a = ys[s] * n.U, b = ys[s] * n.V;
        real f = axi ? FT * b : 0.0;
        const real rx = n.Diff * gx, ry = n.Diff * gy;
        a -= rx;
        b -= ry;
        f = axi ? f - ry : 0.0;
        out->As[o] = a;
        out->Bs[o] = b;
        if (axi) out->Fs[o] = f;
      }
    }
  }
};

// Gradients + FillNode2D + dt + chemistry of one cell into the register node
// `c` (no stores).  Returns the local dt (1.0 when the cell does not limit
// dt); *early: solid / unset node (only S is carried); *filled: fill_node()
// did not skip the node.  `inplace`: the fluxes are updated in place, so
// those of the flow and species equations need not be loaded (fill_node
// rewrites them on every node it does not skip).
// An accessor that declares TILE_TURB is a lean tile's (hip/lean_mech.hpp): it
// supplies the node's thermodynamic state and the mixture closure (IO::mixer),
// names the turbulence-model set of fill_node (TILE_TURB), and fill_compute
// stops after fill_node (no dt, transport or slot fractions: its caller forms
// those once per cell).
template <class IO, class = void>
struct io_is_tile : std::false_type {};
template <class IO>
struct io_is_tile<IO, std::void_t<decltype(IO::TILE_TURB)>> : std::true_type {};
// An accessor that declares TURB_SET names fill_node's turbulence-model set
// (physics.hpp; the lean N-S kernel's k-eps / SST / SA variants).
template <class IO, int DEF, class = void>
struct io_turb_set : std::integral_constant<int, DEF> {};
template <class IO, int DEF>
struct io_turb_set<IO, DEF, std::void_t<decltype(IO::TURB_SET)>> : std::integral_constant<int, IO::TURB_SET> {};

template <int MODE, int NSB, class IO, bool KEPS_ONLY = false>
HF_HD inline real fill_compute(const StepParams& P, IO& io, CellLocal& c, real* mY, real* mgx, real* mgy,
                               const MechData* mech, int nsp, int i, int j, bool inplace, int* neg_T,
                               bool* early, bool* filled_out, const SoA* sout = nullptr) {
  const u64 CT = io.CT();
  constexpr bool MECH = MODE == SK_MECH;
  constexpr bool SGL = MODE == SK_SGL, SG = MODE == SK_SGL || MODE == SK_SGT;
  for (int k = 0; k < NEQ; k++) c.S[k] = sk_live(MODE, k) ? io.S(k) : 0.0;
  *early = false;
  *filled_out = false;
  if (has_all(CT, CT_SOLID) || !has_all(CT, CT_NODE_IS_SET)) {
    *early = true;
    return 1.0;
  }
  const bool active = !has_all(CT, NT_FC);
  const uint8_t gf = io.gf();
  const bool axi = P.fpa.FT != 0;   // F is only read by the axisymmetric predictor
  const bool ns = P.sm == SM_NS;    // turbulence sources live in Src[I_K], Src[I_EPS]
  c.CT = CT;
  c.TurbType = io.TT();
  for (int k = 0; k < NEQ; k++) {
    const bool ld = sk_live(MODE, k);
    // fill_node() rewrites A, B (and F) of the flow and species equations of
    // every node it does not skip, so those are loaded only when the fluxes
    // are not updated in place (fused Euler ping-pong); a skipped node keeps
    // the stored ones (see the store below)
    const bool fld = ld && (!inplace || k >= 4 + NCOMP);
    c.A[k] = fld ? io.A(k) : 0.0;
    c.B[k] = fld ? io.B(k) : 0.0;
    c.F[k] = (axi && fld) ? io.F(k) : 0.0;
    c.Src[k] = (ld && ((k >= 4 + NCOMP && ns) || (gf & GF_SRC))) ? io.Src(k) : 0.0;
    c.SrcAdd[k] = (ld && (gf & GF_SRCADD)) ? io.SrcAdd(k) : 0.0;
    c.RX[k] = c.RY[k] = 0;
  }
  c.U = io.Uo();
  c.V = io.Vo();
  c.Tg = io.To();
  c.p = io.p();
  c.k = io.kk();
  c.R = io.R();
  c.CP = io.CP();
  c.lam = io.lam();
  c.mu = io.mu();
  const bool wall = has_all(CT, CT_WALL_NO_SLIP) || has_all(CT, CT_WALL_LAW);
  if (SGL) {   // recomputed before use, zero, or turbulence/chemistry-only
    c.Diff = c.mu_t = c.lam_t = c.l_min = c.y_plus = c.Re_local = c.Tf = 0.0;
    c.BGX = wall ? io.BGX() : 0.0;
    c.BGY = wall ? io.BGY() : 0.0;
  } else {
    c.Diff = io.Diff();
    c.mu_t = io.mu_t();
    c.lam_t = io.lam_t();
    c.l_min = io.l_min();
    c.y_plus = io.y_plus();
    c.Re_local = io.Re_local();
    c.BGX = io.BGX();
    c.BGY = io.BGY();
    c.Tf = io.Tf();
  }
  c.Uw = c.Vw = 0;
  c.y = (j + 0.5) * P.dy;
  for (int s = 0; s < NSPEC; s++) {
    c.Y[s] = SG ? (s == NCOMP ? 1.0 : 0.0) : io.Y(s);
    c.droYdx[s] = c.droYdy[s] = 0;
  }
  // mechanism species: mass fractions and d(rho Y_s)/dx,y (active viscous nodes)
  if (MECH) {
    const real rho = c.S[I_RHO];
    // species loads at a clamped index, unconditionally: no branch between
    // them, so all NSB loads are in flight together (a guarded load per
    // species was one memory round trip each)
#pragma unroll
    for (int s = 0; s < (MECH ? NSB : 1); s++) {
      const real ys = io.Ys(s < nsp ? s : nsp - 1);
      mY[s] = (s < nsp && rho != 0) ? hf_div(ys, rho) : 0.0;
      mgx[s] = mgy[s] = 0.0;
    }
  }
  if (!(active && ns)) {   // velocity/temperature gradients are recomputed below for active viscous nodes
    c.dUdx = io.grad(G_DUDX);
    c.dUdy = io.grad(G_DUDY);
    c.dVdx = io.grad(G_DVDX);
    c.dVdy = io.grad(G_DVDY);
    c.dTdx = io.grad(G_DTDX);
    c.dTdy = io.grad(G_DTDY);
  }
  if (SGL) {
    c.dkdx = c.dkdy = c.depsdx = c.depsdy = 0.0;
  } else {
    c.dkdx = io.grad(G_DKDX);
    c.dkdy = io.grad(G_DKDY);
    c.depsdx = io.grad(G_DEDX);
    c.depsdy = io.grad(G_DEDY);
  }

  // lazy mechanism gradients (sout): formed in MechMixLazy::heat_flux
  real lz_dx = 0, lz_dy = 0;
  bool lz_nx0 = false, lz_ny0 = false;
  constexpr bool TILE = io_is_tile<IO>::value;
  const bool lazy = MECH && (sout != nullptr || TILE) && P.sm == SM_NS;
  if (active && P.sm == SM_NS) {
    const uint8_t nbm = io.nb();
    const int n1 = (nbm & NB_XL) ? 1 : 0, n2 = (nbm & NB_XR) ? 1 : 0;
    const int n3 = (nbm & NB_YU) ? 1 : 0, n4 = (nbm & NB_YD) ? 1 : 0;
    io.set_nb(i, j, P.ny, n1, n2, n3, n4);
    const real dx_1_n = hf_div(hf_div(1.0, P.dx), (real)(n1 + n2 > 1 ? n1 + n2 : 1));
    const real dy_1_m = hf_div(hf_div(1.0, P.dy), (real)(n3 + n4 > 1 ? n3 + n4 : 1));
    lz_dx = dx_1_n;
    lz_dy = dy_1_m;
    real aR = io.Sn(0, ND_R), aL = io.Sn(0, ND_L), aU = io.Sn(0, ND_U), aD = io.Sn(0, ND_D);
    c.droYdx[NCOMP] = c.droYdy[NCOMP] = 0.;
    const bool nx0 = has_all(CT, CT_dYdx_NULL), ny0 = has_all(CT, CT_dYdy_NULL);
    // SGL: species partial densities are +0, so aR - 0 - 0 - 0 == aR and the
    // species gradients are (0 - 0) * d == +0
    for (int k = 4; k < ((SG || MECH) ? 4 : 4 + NCOMP); k++) {
      if (!nx0) {
        c.droYdx[k - 4] = (io.Sn(k, ND_R) - io.Sn(k, ND_L)) * dx_1_n;
        aR -= io.Sn(k, ND_R);
        aL -= io.Sn(k, ND_L);
      }
      if (!ny0) {
        c.droYdy[k - 4] = (io.Sn(k, ND_U) - io.Sn(k, ND_D)) * dy_1_m;
        aU -= io.Sn(k, ND_U);
        aD -= io.Sn(k, ND_D);
      }
    }
    if (!nx0) c.droYdx[NCOMP] = (aR - aL) * dx_1_n;
    if (!ny0) c.droYdy[NCOMP] = (aU - aD) * dy_1_m;
    lz_nx0 = nx0;
    lz_ny0 = ny0;
    if (MECH && !lazy) {
#pragma unroll
      for (int s = 0; s < (MECH ? NSB : 1); s++) {   // (clamped loads, as above)
        const int sl = s < nsp ? s : nsp - 1;
        const real yR = io.Ysn(sl, ND_R), yL = io.Ysn(sl, ND_L), yU = io.Ysn(sl, ND_U), yD = io.Ysn(sl, ND_D);
        if (s < nsp) {
          if (!nx0) mgx[s] = (yR - yL) * dx_1_n;
          if (!ny0) mgy[s] = (yU - yD) * dy_1_m;
        }
      }
    }
    const real rho = c.S[I_RHO];
    if (has_all(CT, CT_WALL_NO_SLIP) || has_all(CT, CT_WALL_LAW)) {
      c.dUdx = (io.Uon(ND_R) * n1 - io.Uon(ND_L) * n2) * dx_1_n;
      c.dVdx = (io.Von(ND_R) * n1 - io.Von(ND_L) * n2) * dx_1_n;
      c.dUdy = (io.Uon(ND_U) * n3 - io.Uon(ND_D) * n4) * dy_1_m;
      c.dVdy = (io.Von(ND_U) * n3 - io.Von(ND_D) * n4) * dy_1_m;
      if (is_two_eq(c.TurbType)) {
        c.dkdx = (io.Sn(I_K, ND_R) * n1 - io.Sn(I_K, ND_L) * n2) * dx_1_n / rho;
        c.depsdx = (io.Sn(I_EPS, ND_R) * n1 - io.Sn(I_EPS, ND_L) * n2) * dx_1_n / rho;
        c.dkdy = (io.Sn(I_K, ND_U) * n3 - io.Sn(I_K, ND_D) * n4) * dy_1_m / rho;
        c.depsdy = (io.Sn(I_EPS, ND_U) * n3 - io.Sn(I_EPS, ND_D) * n4) * dy_1_m / rho;
      } else if (has_all(c.TurbType, TCT_Spalart_Allmaras_Model)) {
        c.dkdx = (io.Sn(I_K, ND_R) * n1 - io.Sn(I_K, ND_L) * n2) * dx_1_n / rho;
        c.dkdy = (io.Sn(I_K, ND_U) * n3 - io.Sn(I_K, ND_D) * n4) * dy_1_m / rho;
      }
    } else {
      c.dUdx = (io.Uon(ND_R) - io.Uon(ND_L)) * dx_1_n;
      c.dVdx = (io.Von(ND_R) - io.Von(ND_L)) * dx_1_n;
      c.dUdy = (io.Uon(ND_U) - io.Uon(ND_D)) * dy_1_m;
      c.dVdy = (io.Von(ND_U) - io.Von(ND_D)) * dy_1_m;
      if (is_two_eq(c.TurbType)) {
        c.dkdx = hf_div((io.Sn(I_K, ND_R) - io.Sn(I_K, ND_L)) * dx_1_n, rho);
        c.depsdx = hf_div((io.Sn(I_EPS, ND_R) - io.Sn(I_EPS, ND_L)) * dx_1_n, rho);
        c.dkdy = hf_div((io.Sn(I_K, ND_U) - io.Sn(I_K, ND_D)) * dy_1_m, rho);
        c.depsdy = hf_div((io.Sn(I_EPS, ND_U) - io.Sn(I_EPS, ND_D)) * dy_1_m, rho);
      } else if (has_all(c.TurbType, TCT_Spalart_Allmaras_Model)) {
        c.dkdx = hf_div((io.Sn(I_K, ND_R) - io.Sn(I_K, ND_L)) * dx_1_n, rho);
        c.dkdy = hf_div((io.Sn(I_K, ND_U) - io.Sn(I_K, ND_D)) * dy_1_m, rho);
      }
    }
    c.dTdx = (io.Ton(ND_R) - io.Ton(ND_L)) * dx_1_n;
    c.dTdy = (io.Ton(ND_U) - io.Ton(ND_D)) * dy_1_m;
  }

  // P.ffc (NT_FC nodes) differs from P.fpa only in is_mu_t / is_init; patch
  // those two fields rather than binding a runtime-selected reference into the
  // kernel-argument block (which makes the compiler copy StepParams to scratch).
  FillParams fp = P.fpa;
  fp.dt = P.dt;
  if (!active) {
    fp.is_mu_t = P.ffc.is_mu_t;
    fp.is_init = P.ffc.is_init;
  }
  bool filled;
  if constexpr (MECH && TILE) {
    filled = fill_node<CellLocal, typename IO::Mix, IO::TILE_TURB>(
        c, fp, io.mixer(mY, lz_dx, lz_dy, active, lz_nx0, lz_ny0));
  } else if constexpr (MECH) {
    if (lazy) {
      MechMixLazy<NSB, IO> mx{mech, mY, &io, sout, io.N, io.idx, lz_dx, lz_dy, (real)P.fpa.FT, nsp, mech->bath,
                              active, lz_nx0, lz_ny0, P.fpa.FT != 0};
      filled = fill_node(c, fp, mx);
    } else {
      MechMix<NSB> mx{mech, mY, mgx, mgy};
      filled = fill_node(c, fp, mx);
    }
  } else {
    filled = fill_node<CellLocal, RefMix, MODE == SK_SGL ? 0 : io_turb_set<IO, KEPS_ONLY ? 2 : 1>::value>(c, fp);
  }
  *filled_out = filled;
  if constexpr (TILE) return 1.0;

  real dt_local = 1.0;
  if (active) {
    // mechanism mode: the Newton clamps T at MECH_TMIN; reaching it (or NaN)
    // means the energy is unphysical
    if (c.Tg < 0. || (MECH && !(c.Tg > MECH_TMIN))) {
      if (neg_T) *neg_T = 1;
    } else {
      const real AAA = hf_sqrt(c.k * c.R * c.Tg);
      dt_local = P.CFL_min * hf_min(hf_div(P.dx, AAA + std::fabs(c.U)), hf_div(P.dy, AAA + std::fabs(c.V)));
      if (P.visc_cfl > 0 && P.sm == SM_NS) {
        const real nu_eff = (c.mu + c.mu_t) / c.S[I_RHO];
        if (nu_eff > 0) dt_local = hf_min(dt_local, P.visc_cfl / (nu_eff * (1.0 / (P.dx * P.dx) + 1.0 / (P.dy * P.dy))));
      }
      if (MECH) {
        // mixture transport at the new T (the reference's lagged update) and
        // the Tecplot slot fractions
        mech_transport<NSB>(*mech, mY, c.Tg, &c.mu, &c.lam);
        mech_slot_fractions(*mech, mY, c.Y);
      } else if (SG) {
        if (P.chem_model != NO_REACTIONS) chemistry_single_gas_ns(c, *P.species);
      } else {
        if (P.chem_model != NO_REACTIONS) chemistry_zeldovich(c, *P.species, P.sm, P.chem_model);
        if (P.chem_model == CRM_ARRENIUS) chemistry_arrhenius_src(c, *P.species, P.dt);
      }
    }
  }
  return dt_local;
}

template <int MODE = SK_GENERIC, int NSB = 1, bool LAZY = false>
HF_HD inline real fill_cell(const StepParams& P, const SoA& sin, const SoA& prim_old, const SoA& out, int i, int j,
                            int* neg_T, bool store_grad) {
  const long N = sin.N;
  const long idx = (long)i * P.ny + j;
  constexpr bool MECH = MODE == SK_MECH;
  constexpr bool SGL = MODE == SK_SGL, SG = MODE == SK_SGL || MODE == SK_SGT;
  CellLocal c;
  real mY[MECH ? NSB : 1], mgx[MECH ? NSB : 1], mgy[MECH ? NSB : 1];
  FillSoAIO io(sin, prim_old, idx);
  const bool inplace = io.inplace(out);
  bool early, filled;
  const bool lazy = MECH && LAZY && P.sm == SM_NS;
  const real dt_local = fill_compute<MODE, NSB>(P, io, c, mY, mgx, mgy, sin.mech, sin.nsp, i, j, inplace, neg_T,
                                                &early, &filled, lazy ? &out : nullptr);
  if (early) {
    for (int k = 0; k < NEQ; k++)
      if (sk_live(MODE, k)) out.S[k * N + idx] = c.S[k];
    return 1.0;
  }
  const uint8_t gf = io.gf();
  const bool axi = P.fpa.FT != 0;
  const bool ns = P.sm == SM_NS;
  const bool active = !has_all(c.CT, NT_FC);
  // SGL: a skipped node (fill_node returned false) keeps its stored fluxes
  for (int k = 0; k < NEQ; k++) {
    if (!sk_live(MODE, k)) continue;
    out.S[k * N + idx] = c.S[k];
    if (filled || !inplace || k >= 4 + NCOMP) {
      out.A[k * N + idx] = c.A[k];
      out.B[k * N + idx] = c.B[k];
      if (axi) out.F[k * N + idx] = c.F[k];
    }
    if ((k >= 4 + NCOMP && ns) || (gf & GF_SRC)) out.Src[k * N + idx] = c.Src[k];
    if (gf & GF_SRCADD) out.SrcAdd[k * N + idx] = c.SrcAdd[k];
  }
  if (MECH && filled && !lazy) {
    // species fluxes: inviscid, Le = 1 diffusion with Diff (the reference's
    // slot fluxes), axisymmetric F (N-S flat: F = 0)
    const bool nsv = P.sm == SM_NS;
    const int bath = sin.mech->bath, nsp = sin.nsp;
    real ysv[MECH ? NSB : 1];   // loaded together (clamped index), then used
#pragma unroll
    for (int s = 0; s < (MECH ? NSB : 1); s++) ysv[s] = sin.Ys[(long)(s < nsp ? s : nsp - 1) * N + idx];
#pragma unroll
    for (int s = 0; s < (MECH ? NSB : 1); s++) {
      if (s >= nsp) break;
      if (s == bath) continue;
      const long o = (long)s * N + idx;
      const real rys = ysv[s];
      real a = rys * c.U, b = rys * c.V;
      real f = axi ? (real)P.fpa.FT * b : 0.0;
      if (nsv) {
        const real rx = c.Diff * mgx[s], ry = c.Diff * mgy[s];
        a -= rx;
        b -= ry;
        f = axi ? f - ry : 0.0;
      }
      out.As[o] = a;
      out.Bs[o] = b;
      if (axi) out.Fs[o] = f;
    }
  }
  out.U[idx] = c.U;
  out.V[idx] = c.V;
  out.Tg[idx] = c.Tg;
  out.p[idx] = c.p;
  out.kk[idx] = c.k;
  if (!SG) out.R[idx] = c.R;   // single gas: R_air, never changes
  out.CP[idx] = c.CP;
  out.lam[idx] = c.lam;
  out.mu[idx] = c.mu;
  if (!SGL || store_grad) out.Diff[idx] = c.Diff;
  if (!SGL) {
    out.mu_t[idx] = c.mu_t;
    out.lam_t[idx] = c.lam_t;
    out.Re_local[idx] = c.Re_local;
  }
  // (mechanism mode: the slot fractions are Tecplot output only -- a fill reads
  // them for the slot equations' wall sources, which are not live -- so they
  // are stored on output steps, like the gradients)
  if (!SG && (!MECH || store_grad))
    for (int s = 0; s < NSPEC; s++) out.Y[s * N + idx] = c.Y[s];
  if (store_grad && active && P.sm == SM_NS) {
    out.grad[G_DUDX * N + idx] = c.dUdx;
    out.grad[G_DUDY * N + idx] = c.dUdy;
    out.grad[G_DVDX * N + idx] = c.dVdx;
    out.grad[G_DVDY * N + idx] = c.dVdy;
    out.grad[G_DTDX * N + idx] = c.dTdx;
    out.grad[G_DTDY * N + idx] = c.dTdy;
  }
  if (!SGL && store_grad && active && P.sm == SM_NS) {   // turbulence gradients (never read by SGL)
    out.grad[G_DKDX * N + idx] = c.dkdx;
    out.grad[G_DKDY * N + idx] = c.dkdy;
    out.grad[G_DEDX * N + idx] = c.depsdx;
    out.grad[G_DEDY * N + idx] = c.depsdy;
  }
  return dt_local;
}

// Operator-split kinetics of one cell (mechanism mode): the predicted species
// mid.Ys -> out.Ys at constant rho and e over the step's dt.  Inactive
// cells, cells colder than MechData::Tchem (by the previous step's T) and
// dt = 0 copy through.  Runtime mechanism data: the host path of the device
// kernels (chem_fast.hip / chem_mech.hip).
template <int NSB>
HF_HD inline void mech_chem_soa_cell(const StepParams& P, const SoA& mid, const SoA& out, const real* Tprev, int i,
                                     int j) {
  const long N = mid.N;
  const long idx = (long)i * P.ny + j;
  const MechData& m = *mid.mech;
  const real rho = mid.S[idx];
  const bool react = is_active(mid.CT[idx]) && rho > 0 && Tprev[idx] >= m.Tchem && P.dt > 0;
  real rhoY[NSB];
#pragma unroll
  for (int s = 0; s < NSB; s++) rhoY[s] = s < m.ns ? mid.Ys[(long)s * N + idx] : 0.0;
  if (react) {
    const real ru = mid.S[(long)I_RHOU * N + idx], rv = mid.S[(long)I_RHOV * N + idx];
    const real e = (mid.S[(long)I_RHOE * N + idx] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
    real T = Tprev[idx];
    mech_chem_cell<NSB>(m, rho, e, rhoY, &T, P.dt, m.nsub);
  }
#pragma unroll
  for (int s = 0; s < NSB; s++)
    if (s < m.ns) out.Ys[(long)s * N + idx] = rhoY[s];
}

}  // namespace hf2d

namespace hf2d {

// ---------------------------------------------------------------------------
// Wall heat sources, owner-computes form of CalcHeatOnWallSources
// (deeps2d_core.cpp:2679-2833).  The reference visits wall cells column by
// column (i outer, j inner) and, per wall cell, its solid neighbours in the
// order Down, Up, Left, Right, updating the solid's Q_conv in place.  A solid
// cell therefore sees its wall neighbours in the order (i-1,j), (i,j-1),
// (i,j+1), (i+1,j); we replay that sequence per solid cell and record the
// Q value after each update in qdir[d] so that the wall cell can pick it up.
// qdir slots: 0 = updated by the left wall cell, 1 = by the lower, 2 = by the
// upper, 3 = by the right wall cell.
// ---------------------------------------------------------------------------
HF_HD inline bool is_wall_gas(u64 ct) {
  return !has_all(ct, CT_SOLID) && (has_all(ct, CT_WALL_LAW) || has_all(ct, CT_WALL_NO_SLIP));
}

HF_HD inline void wall_heat_solid_cell(const StepParams& P, const SoA& s, real* qdir, int i, int j) {
  const long N = s.N;
  const long idx = (long)i * P.ny + j;
  for (int d = 0; d < 4; d++) qdir[d * N + idx] = 0.;
  if (!has_all(s.CT[idx], CT_SOLID)) return;
  real Q = 0.;
  const real Ts = s.Tg[idx];
  const int di[4] = {-1, 0, 0, 1};
  const int dj[4] = {0, -1, 1, 0};
  for (int d = 0; d < 4; d++) {
    const int wi = i + di[d], wj = j + dj[d];
    if (wi < 0 || wj < 0 || wi >= P.nx || wj >= P.ny) continue;
    const long w = (long)wi * P.ny + wj;
    if (!is_wall_gas(s.CT[w])) continue;
    const real h = (d == 0 || d == 3) ? P.dx : P.dy;
    const real lam_eff = s.lam[w] + s.lam_t[w];
    if (Q > 0.)
      Q = (Q - lam_eff * (Ts - s.Tg[w]) / h) * 0.5;
    else
      Q = -lam_eff * (Ts - s.Tg[w]) / h;
    qdir[d * N + idx] = Q;
  }
  s.Q_conv[idx] = Q;
}

HF_HD inline void wall_heat_wall_cell(const StepParams& P, const SoA& s, const real* qdir, int i, int j) {
  const long N = s.N;
  const long idx = (long)i * P.ny + j;
  if (!is_wall_gas(s.CT[idx])) return;
  real* srcE = s.SrcAdd + (long)I_RHOE * N;
  // Down, Up, Left, Right: later assignments overwrite earlier ones.
  if (j > 0 && has_all(s.CT[idx - 1], CT_SOLID)) srcE[idx] = -P.dt * qdir[2 * N + idx - 1] / P.dy;
  if (j < P.ny - 1 && has_all(s.CT[idx + 1], CT_SOLID)) srcE[idx] = -P.dt * qdir[1 * N + idx + 1] / P.dy;
  if (i > 0 && has_all(s.CT[idx - P.ny], CT_SOLID)) srcE[idx] = -P.dt * qdir[3 * N + idx - P.ny] / P.dx;
  if (i < P.nx - 1 && has_all(s.CT[idx + P.ny], CT_SOLID)) srcE[idx] = -P.dt * qdir[0 * N + idx + P.ny] / P.dx;
}

// y+ from the friction velocity of the nearest wall node (the MPI build's
// per-cycle ParallelRecalc_y_plus, deeps2d_core.cpp:2291-2322, in O(N) form):
// the owner of each wall node forms its friction velocity, the values of all
// strips are merged (SolverBase::merge_wall_uw), then every cell takes its
// wall's -- a cell whose wall lies in another strip sees that strip's value.
HF_HD inline real wall_friction_velocity(const SoA& s, long w) {
  const long N = s.N;
  const real tau_w = (std::fabs(s.grad[G_DUDY * N + w]) + std::fabs(s.grad[G_DVDX * N + w])) * s.mu[w];
  return std::sqrt(tau_w / s.S[w] + 1e-30);
}
HF_HD inline void y_plus_apply(const SoA& s, long idx, const real* uw, const uint8_t* uw_ok) {
  const u64 ct = s.CT[idx];
  if (!has_all(ct, CT_NODE_IS_SET) || has_all(ct, CT_SOLID)) return;
  const int k = s.wslot[idx];
  if (k < 0 || !uw_ok[k]) return;
  s.y_plus[idx] = std::fabs(uw[k] * s.l_min[idx] * s.S[idx] / s.mu[idx]);
}

}  // namespace hf2d
