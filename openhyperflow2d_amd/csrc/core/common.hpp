// hf2d — MI355X-native 2D compressible reacting-flow solver.
// Common definitions shared by host code (g++/amdclang++) and HIP device code.
//
// Condition-flag bit values, equation indices and the checkpoint record layout
// are part of the on-disk/deck compatibility contract with OpenHyperFLOW2D
// (reference: libOpenHyperFLOW2D/hyper_flow_node.hpp:53-128,
//  hyper_flow_turbulence.hpp:17-99), so they keep the reference's numbering.
#pragma once

#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HF_HD __host__ __device__
#define HF_DEV __device__
#else
#define HF_HD
#define HF_DEV
#endif

namespace hf2d {

#ifdef HF2D_FP32
using real = float;   // FP32 build option (host CLI hf2d_cpu_fp32; the reference's -DFP=float)
#else
using real = double;   // FP64 default (the reference's FP_OPTS = -DFP=double, gcc.compiler:22)
#endif
using u64 = std::uint64_t;


// ---------------------------------------------------------------------------
// Species / equation layout (NUM_COMPONENTS = 3 additional species + inert).
// ---------------------------------------------------------------------------
constexpr int NCOMP = 3;               // additional components (fuel, ox, cp)
constexpr int NSPEC = NCOMP + 1;       // + inert (air)
constexpr int NEQ = 6 + NCOMP;         // rho, rhoU, rhoV, rhoE, rhoY[3], k, eps
constexpr int I_RHO = 0, I_RHOU = 1, I_RHOV = 2, I_RHOE = 3;
constexpr int I_YFU = 4, I_YOX = 5, I_YCP = 6;
constexpr int I_K = 7, I_NUT = 7, I_EPS = 8, I_OMEGA = 8;
constexpr int H_FU = 0, H_OX = 1, H_CP = 2, H_AIR = 3;

// ---------------------------------------------------------------------------
// Cell condition bits (CT word, 64 bit).
// ---------------------------------------------------------------------------
enum : u64 {
  CT_NO_COND = 0x0,
  CT_Rho_CONST = 0x01,
  CT_U_CONST = 0x02,
  CT_V_CONST = 0x04,
  CT_T_CONST = 0x08,
  CT_Y_CONST = 0x010,
  CT_dRhodx_NULL = 0x020,
  CT_dUdx_NULL = 0x040,
  CT_dVdx_NULL = 0x080,
  CT_dTdx_NULL = 0x0100,
  CT_dYdx_NULL = 0x0200,
  CT_dRhody_NULL = 0x0400,
  CT_dUdy_NULL = 0x0800,
  CT_dVdy_NULL = 0x01000,
  CT_dTdy_NULL = 0x02000,
  CT_dYdy_NULL = 0x04000,
  CT_d2Rhodx2_NULL = 0x08000,
  CT_d2Udx2_NULL = 0x010000,
  CT_d2Vdx2_NULL = 0x020000,
  CT_d2Tdx2_NULL = 0x040000,
  CT_d2Ydx2_NULL = 0x080000,
  CT_d2Rhody2_NULL = 0x0100000,
  CT_d2Udy2_NULL = 0x0200000,
  CT_d2Vdy2_NULL = 0x0400000,
  CT_d2Tdy2_NULL = 0x0800000,
  CT_d2Ydy2_NULL = 0x01000000,
  CT_NONREFLECTED = 0x02000000,
  CT_WALL_NO_SLIP = 0x04000000,
  CT_WALL_LAW = 0x08000000,
  CT_GAS = 0x010000000,
  CT_BL_REFINEMENT = 0x020000000,
  CT_SOLID = 0x040000000,
  CT_NODE_IS_SET = 0x080000000,
  CT_LIQUID = 0x0100000000ULL,
  CT_TIME_DEPEND = 0x0200000000ULL,
};

// Macro node types (combinations of CT bits).
enum : u64 {
  NT_FC = CT_Rho_CONST | CT_U_CONST | CT_V_CONST | CT_Y_CONST | CT_T_CONST | CT_NODE_IS_SET,
  NT_D0X = CT_NODE_IS_SET | CT_dRhodx_NULL | CT_dUdx_NULL | CT_dVdx_NULL | CT_dTdx_NULL | CT_dYdx_NULL,
  NT_D2X = CT_NODE_IS_SET | CT_d2Rhodx2_NULL | CT_d2Udx2_NULL | CT_d2Vdx2_NULL | CT_d2Tdx2_NULL |
           CT_d2Ydx2_NULL,
  NT_D0Y = CT_NODE_IS_SET | CT_dRhody_NULL | CT_dUdy_NULL | CT_dVdy_NULL | CT_dTdy_NULL | CT_dYdy_NULL,
  NT_D2Y = CT_NODE_IS_SET | CT_d2Rhody2_NULL | CT_d2Udy2_NULL | CT_d2Vdy2_NULL | CT_d2Tdy2_NULL |
           CT_d2Ydy2_NULL,
  NT_AY = CT_NODE_IS_SET | NT_D0X | CT_U_CONST,
  NT_AX = CT_NODE_IS_SET | NT_D0Y | CT_V_CONST,
  NT_WALL_LAW = CT_NODE_IS_SET | CT_WALL_LAW,
  NT_WNS = CT_NODE_IS_SET | CT_WALL_NO_SLIP | CT_U_CONST | CT_V_CONST,
  NT_S = CT_SOLID | CT_NODE_IS_SET,
  // The reference defines NT_F_2D as (!CT_SOLID | NODE_IS_SET) which is just
  // NODE_IS_SET (logical not of a non-zero constant); kept for compatibility.
  NT_F = CT_NODE_IS_SET,
  NT_FC_TIME_DEPEND = NT_FC | CT_TIME_DEPEND,
  NT_FARFIELD = NT_FC | CT_NONREFLECTED,
};
// wall node directions into the flow (Case::wall_dirs, Config::WallBlendCells)
enum : uint8_t { WD_XP = 1, WD_XM = 2, WD_YP = 4, WD_YM = 8 };

// Turbulence condition bits (TurbType word).
enum : u64 {
  TCT_No_Turbulence = 0x0,
  TCT_k_CONST = 0x01,
  TCT_eps_CONST = 0x02,
  TCT_dkdx_NULL = 0x04,
  TCT_depsdx_NULL = 0x08,
  TCT_dkdy_NULL = 0x010,
  TCT_depsdy_NULL = 0x020,
  TCT_d2kdx2_NULL = 0x040,
  TCT_d2epsdx2_NULL = 0x080,
  TCT_d2kdy2_NULL = 0x0100,
  TCT_d2epsdy2_NULL = 0x0200,
  TCT_k_eps_Model = 0x0400,
  TCT_Prandtl_Model = 0x0800,
  TCT_Integral_Model = 0x01000,
  TCT_eps_mud2kdx2_WALL = 0x02000,
  TCT_eps_mud2kdy2_WALL = 0x04000,
  TCT_eps_Cmk2kXn_WALL = 0x08000,
  TCT_Spalart_Allmaras_Model = 0x010000,
  TCT_k_omega_Model = 0x020000,
  TCT_k_omega_SST_Model = 0x040000,
  TCT_Baldwin_Lomax_Model = 0x080000,
  TCT_nut_92_Model = 0x0100000,
  TCT_Smagorinsky_Model = 0x0200000,
};
constexpr u64 TCT_nu_t_CONST = TCT_k_CONST;

enum TurbExtModel : int {
  TEM_Prandtl = 0,
  TEM_vanDriest,
  TEM_Escudier,
  TEM_Klebanoff,
  TEM_k_eps_Std,
  TEM_k_eps_Chien,
  TEM_k_eps_JL,
  TEM_k_eps_LSY,
  TEM_k_eps_RNG,
  TEM_k_eps_Realisable,
  TEM_Spalart_Allmaras,
  TEM_Baldwin_Lomax,
  TEM_nut_92_Sekundov,
  TEM_k_omega_Wilcox,
  TEM_k_omega_SST,
  TEM_Smagorinsky,
};

enum SolverMode : int { SM_EULER = 0, SM_NS = 1 };
enum FlowType : int { FT_FLAT = 0, FT_AXISYMMETRIC = 1 };
enum BlendingFactorFunction : int {
  BFF_L = 0, BFF_LR, BFF_S, BFF_SR, BFF_SQR, BFF_SQRR,
  BFF_MACH, BFF_LG, BFF_MIXED, BFF_HYBRID, BFF_SQR_PRESSURE, BFF_SR_LIMITED
};
enum ChemModel : int { NO_REACTIONS = 0, CRM_ZELDOVICH = 1, CRM_ARRENIUS = 2, CRM_EDM = 3 };

HF_HD inline bool has_all(u64 word, u64 mask) { return (word & mask) == mask; }

// ---------------------------------------------------------------------------
// CellRecord: byte-compatible with the reference's FlowNode2D<double,3>
// (1248 bytes, x-major file order). Used on the host for pre-processing, the
// reference-order CPU oracle and the .hf2d checkpoint.  Field order matters.
// ---------------------------------------------------------------------------
struct CellRecord {
  // FlowNodeCore2D
  real S[NEQ];
  real dSdx[NEQ];
  real dSdy[NEQ];
  // FlowNodeTurbulence2D
  u64 TurbType;
  real l_min, y_plus, Re_local, mu_t, lam_t;
  real dkdx, dkdy, depsdx, depsdy;
  // FlowNode2D
  real x, y;
  int32_t ix, iy;
  u64 nb_ptr[4];  // Up/Down/Left/Right node pointers: never set (always 0)
  real p;
  int32_t idXl, idYu, idXr, idYd;
  int32_t NGX, NGY;
  u64 CT;
  int32_t i_wall, j_wall;
  real beta[NEQ];
  real Q_conv;
  real time;
  real k, R, lam, mu, CP, Diff;
  real Tf;
  real A[NEQ], B[NEQ], F[NEQ], RX[NEQ], RY[NEQ], Src[NEQ], SrcAdd[NEQ];
  real Tg, U, V, Y[NSPEC];
  real Uw, Vw;
  real droYdx[NSPEC], droYdy[NSPEC];
  real dUdx, dUdy, dVdx, dVdy, dTdx, dTdy;
  real BGX, BGY;

  HF_HD bool is(u64 mask) const { return (CT & mask) == mask; }
  HF_HD bool is_turb(u64 mask) const { return (TurbType & mask) == mask; }
};

// (FP64: the reference's 1248-byte record; the FP32 build writes the float
// layout of the reference's -DFP=float build, whose checkpoints are not
// interchangeable with FP64 ones either)
#ifndef HF2D_FP32
static_assert(sizeof(CellRecord) == 1248, "CellRecord must match the 1248-byte .hf2d record");
static_assert(offsetof(CellRecord, TurbType) == 216, "layout");
static_assert(offsetof(CellRecord, x) == 296, "layout");
static_assert(offsetof(CellRecord, p) == 352, "layout");
static_assert(offsetof(CellRecord, CT) == 384, "layout");
static_assert(offsetof(CellRecord, beta) == 400, "layout");
static_assert(offsetof(CellRecord, A) == 544, "layout");
static_assert(offsetof(CellRecord, Tg) == 1048, "layout");
static_assert(offsetof(CellRecord, Y) == 1072, "layout");
static_assert(offsetof(CellRecord, droYdx) == 1120, "layout");
static_assert(offsetof(CellRecord, dUdx) == 1184, "layout");
static_assert(offsetof(CellRecord, BGX) == 1232, "layout");
#endif

// ---------------------------------------------------------------------------
// Correctly rounded FP64 division and square root for operands of ordinary
// magnitude.  The compiler's IEEE expansion on gfx950 wraps the Newton-
// Raphson / Markstein sequence in v_div_scale (operand scaling near the
// exponent limits) and v_div_fixup (inf / nan / zero cases), 11 VALU
// instructions per division; for operands whose exponents are far from the
// limits the scaling is the identity and the fixup returns the quotient
// unchanged, so the bare sequence (8 instructions) yields the same correctly
// rounded result, bit for bit -- the host computes a / b.  v_div_fixup is
// kept (9 instructions), so zero, infinite and NaN operands still give the
// IEEE result; only operands within ~2^100 of the exponent limits, where the
// scaling would engage, can differ.  hf_sqrt keeps the
// zero / +inf case (a steady cell has a zero residual) and drops the tiny-
// argument scaling (inputs >= 2^-767 or exactly 0).
// ---------------------------------------------------------------------------
HF_HD inline double hf_div(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(b);
  double t = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, t, r);
  t = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, t, r);
  const double q = a * r;
  const double e = __builtin_fma(-b, q, a);
  // v_div_fixup: zero / inf / nan operands give the IEEE result
  return __builtin_amdgcn_div_fixup(__builtin_fma(e, r, q), b, a);
#else
  return a / b;
#endif
}
HF_HD inline double hf_sqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return (x == 0.0 || x == __builtin_inf()) ? x : g;
#else
  return __builtin_sqrt(x);
#endif
}

// Piecewise-linear property table with the reference's rule: linear
// interpolation inside, linear *extrapolation* from the end segment outside
// (obj_data/obj_data.cpp:1822-1859).  Plain-old-data so it can live in device
// constant/global memory.
constexpr int MAX_TABLE_PTS = 64;
// (double in every build: deck tables also carry the contour / area
// coordinates, which the FP32 build converts to cell indices in double)
struct TableData {
  int n = 0;
  double x[MAX_TABLE_PTS];
  double y[MAX_TABLE_PTS];
};

HF_HD inline real table_eval(const TableData& t, real xv) {
  const int n = t.n;
  if (n <= 0) return 0.0;
  if (n == 1) return t.y[0];
  int i;
  if (xv <= t.x[0]) {
    i = 1;
  } else if (xv >= t.x[n - 1]) {
    i = n - 1;
  } else {
    for (i = 1; i < n; i++)
      if (xv >= t.x[i - 1] && xv < t.x[i]) break;
  }
  return t.y[i] + hf_div((t.y[i - 1] - t.y[i]) * (xv - t.x[i]), t.x[i - 1] - t.x[i]);
}

// Species property pack: R, formation enthalpy and Cp/lam/mu(T) tables for
// fuel, oxidizer, combustion products and inert gas.
struct SpeciesProps {
  real K0 = 0, gamma = 0, Tf = 0;
  real R[NSPEC] = {0, 0, 0, 0};   // fu, ox, cp, air
  real H[NSPEC] = {0, 0, 0, 0};
  TableData Cp[NSPEC];
  TableData lam[NSPEC];
  TableData mu[NSPEC];
  // finite-rate global reaction 2 fu + ox -> 2 cp (new, ChemicalReactionsModel=2):
  // W = A exp(-Ta/T) [fu]^a [ox]^b  [mol/m^3/s], concentrations in mol/m^3
  real arr_A = 1.8e10, arr_Ta = 17614.0, arr_a = 1.0, arr_b = 0.5;
  real M[NSPEC] = {0, 0, 0, 0};   // molar masses from R_s (kg/mol)
};

}  // namespace hf2d
