// K12 kinetics of a compiled mechanism, device side (no includes besides
// chem_fast_types.hpp): the per-cell integrator and the kernel bodies.
// Included by chem_fast.hip for the built-in mechanisms and handed to hiprtc
// with a generated mechanism struct for any mechanism loaded from a file
// (chem_rtc.hip), so both run the same code.
//
// Same algorithm as the runtime-data host integrator mech_chem_cell
// (core/mechanism.hpp), which is its oracle: nsub linearised backward-Euler
// substeps (I - h J) dc = h w(c, T) at constant rho and e, reversible rates from
// the NASA-7 equilibrium constants, third-body efficiencies, Troe fall-off,
// c <- max(c + dc, 0), mass re-normalised, T re-solved from e (Newton).
//
// Why VALU and not MFMA here: on CDNA4 the FP64 matrix rate equals the FP64
// vector rate, and the stoichiometric matrix of H2/air is ~20 % dense, so the
// per-cell dense J = N D product the MFMA kernel (chem_mech.hip) issues does 5-10x
// the FLOPs of this kernel's sparse accumulation.  Here the mechanism is a
// template parameter: every reaction is a separate instantiation, all species
// indices are compile-time constants, the 9x10 system of a cell lives in VGPRs
// and only the non-zero Jacobian entries are accumulated.
#pragma once

#include "chem_fast_types.hpp"

namespace hf2d {
namespace chemk {

constexpr double RU = 8.314462618, PATM = 101325.0, TMIN = 20.0, TMAX = 6000.0, TLO = 200.0;   // mechanism.hpp MECH_*

template <int... Is>
struct IntSeq {};
template <int N, int... Is>
struct MakeSeqImpl : MakeSeqImpl<N - 1, N - 1, Is...> {};
template <int... Is>
struct MakeSeqImpl<0, Is...> {
  using type = IntSeq<Is...>;
};
template <int N>
using MakeSeq = typename MakeSeqImpl<N>::type;

// Kernel arguments of the kinetics pass (plain pointers: the hiprtc kernels
// share no structs with the solver).  dt is the device dt slot of the step.
struct ChemArgs {
  const double* S;               // conserved state [NEQ * N] (rho, rhoU, rhoV, rhoE used)
  const double* Yin;             // predicted species [ns * N]
  double* Yout;                  // post-kinetics species
  const double* Tprev;           // T of the last fill (Newton guess, reaction threshold)
  const unsigned long long* CT;  // node flags
  const unsigned long long* dt_bits;
  long N, c0, c1;
  double Tchem;
  int nsub;
  unsigned long long set_bit, solid_bit, fc_bits;   // CT_NODE_IS_SET, CT_SOLID, NT_FC
  int* list;                     // compacted form: reacting cells
  unsigned* count;
};

__device__ inline double args_dt(const ChemArgs& a) { return __longlong_as_double((long long)*a.dt_bits); }
__device__ inline bool args_active(const ChemArgs& a, unsigned long long ct) {
  return (ct & a.set_bit) == a.set_bit && (ct & a.solid_bit) != a.solid_bit && (ct & a.fc_bits) != a.fc_bits;
}

template <int N>
__device__ __forceinline__ double ipw(double x) {
  if constexpr (N == 1) return x;
  else if constexpr (N == 2) return x * x;
  else if constexpr (N == 3) return x * x * x;
  else return 1.0;
}

template <class M>
__device__ __forceinline__ const double* coef(int s, double T) {
  return M::a[s][T < M::Tmid[s] ? 0 : 1];
}

// e, cv of the concentrations c at T (per unit mass: divided by rho)
// (below TLO: constant-cp extrapolation, as mech_mix_thermo)
template <class M>
__device__ __forceinline__ void mix_e_cv(const double* c, double rho, double Tin, double* e, double* cv) {
  double se = 0.0, scv = 0.0;
  const double T = Tin < TLO ? TLO : Tin;
#pragma unroll
  for (int s = 0; s < M::NS; s++) {
    const double* a = coef<M>(s, T);
    const double cpR = a[0] + T * (a[1] + T * (a[2] + T * (a[3] + T * a[4])));
    const double hRT = a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2))) +
                       a[5] / T;
    // c_s W_s / rho * (RU / W_s) = c_s RU / rho
    se += c[s] * (T * (hRT - 1.0));
    scv += c[s] * (cpR - 1.0);
  }
  se += scv * (Tin - T);   // (+0 for Tin >= TLO)
  *e = se * RU / rho;
  *cv = scv * RU / rho;
}

template <class M>
__device__ double T_from_e(const double* c, double rho, double e, double T0) {
  double T = T0 > TMIN ? (T0 < TMAX ? T0 : TMAX) : TMIN;
  for (int it = 0; it < 30; it++) {
    double ee, cv;
    mix_e_cv<M>(c, rho, T, &ee, &cv);
    double dT = (e - ee) / cv;
    dT = dT > 500.0 ? 500.0 : (dT < -500.0 ? -500.0 : dT);
    double Tn = T + dT;
    Tn = Tn > TMIN ? (Tn < TMAX ? Tn : TMAX) : TMIN;
    const double d = Tn - T;
    T = Tn;
    if (fabs(d) <= 1e-10 * T) break;
  }
  return T;
}

// Species that appear in no reaction (an inert bath gas such as N2: only a
// collision partner) have a zero production rate, so their row of I - h J is
// the identity row and their solution component is 0 / 1 = +0; their column
// (third-body efficiencies) then only ever multiplies that zero, and the
// elimination never pivots on their row (its other entries are zero).  The
// system is therefore solved over the reacting species alone -- bit for bit
// the same increments, and 9 x 10 -> 8 x 9 doubles of registers for H2 / air.
template <class M>
struct Reacting {
  struct Map {
    int ix[M::NS];
    int n;
  };
  static constexpr Map make() {
    Map m{};
    m.n = 0;
    for (int s = 0; s < M::NS; s++) {
      bool in = false;
      for (int r = 0; r < M::NR; r++) {
        for (int t = 0; t < M::rx[r].nrs; t++) in = in || M::rx[r].rs[t] == s;
        for (int t = 0; t < M::rx[r].nps; t++) in = in || M::rx[r].ps[t] == s;
      }
      m.ix[s] = in ? m.n++ : -1;
    }
    return m;
  }
  static constexpr Map map = make();
  static constexpr int N = map.n;
};

// One reaction's contribution to the augmented system A = [I - h J | h w]
// over the reacting species (Reacting<M>::map.ix: row / column of species s).
template <class M, int R>
__device__ __forceinline__ void apply_rx(const double* c, const double* g, double T, double lnT, double invT,
                                         double lnP0RT, double h, double (&A)[Reacting<M>::N][Reacting<M>::N + 1]) {
  constexpr CRx r = M::rx[R];
  constexpr int NS = M::NS;
  constexpr int NA = Reacting<M>::N;
  constexpr auto X = Reacting<M>::map;
  double kf;
  if constexpr (r.b == 0.0 && r.Ta == 0.0)
    kf = r.A;
  else
    kf = r.A * exp(r.b * lnT - r.Ta * invT);
  double Mc = 1.0;
  if constexpr (r.tb || r.fo) {
    Mc = 0.0;
#pragma unroll
    for (int s = 0; s < NS; s++) Mc += (r.eff >= 0 ? M::eff[r.eff >= 0 ? r.eff : 0][s] : 1.0) * c[s];
  }
  double mult = 1.0;
  if constexpr (r.fo) {
    const double k0 = r.A0 * exp(r.b0 * lnT - r.Ta0 * invT);
    const double Pr = k0 * Mc / kf;
    double F = 1.0;
    if constexpr (r.ntroe >= 3) {
      double Fc = (1.0 - r.troe[0]) * exp(-T / r.troe[1]) + r.troe[0] * exp(-T / r.troe[2]);
      if constexpr (r.ntroe > 3) Fc += exp(-r.troe[3] * invT);
      const double lFc = log10(Fc > 1e-300 ? Fc : 1e-300);
      const double lPr = log10(Pr > 1e-300 ? Pr : 1e-300);
      const double cc = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;
      const double f1 = (lPr + cc) / (nn - 0.14 * (lPr + cc));
      F = pow(10.0, lFc / (1.0 + f1 * f1));
    }
    kf = kf * (Pr / (1.0 + Pr)) * F;
  } else if constexpr (r.tb) {
    mult = Mc;
  }
  double kr = 0.0;
  if constexpr (r.rev) {
    double sg = 0.0;
#pragma unroll
    for (int t = 0; t < r.nps; t++) sg += r.pn[t] * g[r.ps[t]];
#pragma unroll
    for (int t = 0; t < r.nrs; t++) sg -= r.rn[t] * g[r.rs[t]];
    kr = kf * exp(sg - r.dnu * lnP0RT);   // kf / Kc
  }
  // concentration products and their partial derivatives
  double pf = 1.0, pr = 1.0;
#pragma unroll
  for (int t = 0; t < r.nrs; t++) pf *= (r.rn[t] == 1 ? c[r.rs[t]] : (r.rn[t] == 2 ? c[r.rs[t]] * c[r.rs[t]] : c[r.rs[t]] * c[r.rs[t]] * c[r.rs[t]]));
#pragma unroll
  for (int t = 0; t < r.nps; t++) pr *= (r.pn[t] == 1 ? c[r.ps[t]] : (r.pn[t] == 2 ? c[r.ps[t]] * c[r.ps[t]] : c[r.ps[t]] * c[r.ps[t]] * c[r.ps[t]]));
  const double net = kf * pf - kr * pr;
  const double hq = h * mult * net;
#pragma unroll
  for (int t = 0; t < r.nrs; t++) A[X.ix[r.rs[t]]][NA] -= r.rn[t] * hq;
#pragma unroll
  for (int t = 0; t < r.nps; t++) A[X.ix[r.ps[t]]][NA] += r.pn[t] * hq;
  // -h nu_i D_j, D_j = dq/dc_j (j: species index; inert columns dropped)
  auto put = [&](int j, double Dj) {
    const int jj = X.ix[j];
    if (jj < 0) return;
#pragma unroll
    for (int t = 0; t < r.nrs; t++) A[X.ix[r.rs[t]]][jj] += r.rn[t] * h * Dj;
#pragma unroll
    for (int t = 0; t < r.nps; t++) A[X.ix[r.ps[t]]][jj] -= r.pn[t] * h * Dj;
  };
#pragma unroll
  for (int t = 0; t < r.nrs; t++) {
    const int sj = r.rs[t];
    double d = kf * r.rn[t] * (r.rn[t] == 1 ? 1.0 : (r.rn[t] == 2 ? c[sj] : c[sj] * c[sj]));
#pragma unroll
    for (int u = 0; u < r.nrs; u++)
      if (u != t) d *= (r.rn[u] == 1 ? c[r.rs[u]] : (r.rn[u] == 2 ? c[r.rs[u]] * c[r.rs[u]] : c[r.rs[u]] * c[r.rs[u]] * c[r.rs[u]]));
    put(sj, mult * d);
  }
  if constexpr (r.rev) {
#pragma unroll
    for (int t = 0; t < r.nps; t++) {
      const int sj = r.ps[t];
      double d = kr * r.pn[t] * (r.pn[t] == 1 ? 1.0 : (r.pn[t] == 2 ? c[sj] : c[sj] * c[sj]));
#pragma unroll
      for (int u = 0; u < r.nps; u++)
        if (u != t) d *= (r.pn[u] == 1 ? c[r.ps[u]] : (r.pn[u] == 2 ? c[r.ps[u]] * c[r.ps[u]] : c[r.ps[u]] * c[r.ps[u]] * c[r.ps[u]]));
      put(sj, -mult * d);
    }
  }
  if constexpr (r.tb && !r.fo) {
#pragma unroll
    for (int j = 0; j < NS; j++) put(j, (r.eff >= 0 ? M::eff[r.eff >= 0 ? r.eff : 0][j] : 1.0) * net);
  }
}

template <class M, int... Rs>
__device__ __forceinline__ void apply_all(IntSeq<Rs...>, const double* c, const double* g, double T,
                                          double lnT, double invT, double lnP0RT, double h,
                                          double (&A)[Reacting<M>::N][Reacting<M>::N + 1]) {
  (apply_rx<M, Rs>(c, g, T, lnT, invT, lnP0RT, h, A), ...);
}

// Gaussian elimination with partial pivoting; row swaps are selects so the
// matrix stays in registers.  Solution left in A[i][NS].  False if singular.
template <int NS>
__device__ __forceinline__ bool solve(double (&A)[NS][NS + 1]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < NS; k++) {
    int p = k;
    double best = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < NS; i++) {
      const double v = fabs(A[i][k]);
      if (v > best) {
        best = v;
        p = i;
      }
    }
    ok = ok && best > 0.0;
#pragma unroll
    for (int i = k + 1; i < NS; i++) {
      const bool sw = i == p;
#pragma unroll
      for (int j = k; j <= NS; j++) {
        const double t = A[k][j];
        A[k][j] = sw ? A[i][j] : t;
        A[i][j] = sw ? t : A[i][j];
      }
    }
    const double inv = 1.0 / A[k][k];
#pragma unroll
    for (int i = k + 1; i < NS; i++) {
      const double f = A[i][k] * inv;
#pragma unroll
      for (int j = k + 1; j <= NS; j++) A[i][j] -= f * A[k][j];
    }
  }
#pragma unroll
  for (int i = NS - 1; i >= 0; i--) {
    double s = A[i][NS];
#pragma unroll
    for (int j = i + 1; j < NS; j++) s -= A[i][j] * A[j][NS];
    A[i][NS] = s / A[i][i];
  }
  return ok;
}

template <class M>
__device__ void chem_cell(double rho, double e, double* y, double* Tio, double dt, int nsub) {
  constexpr int NS = M::NS;
  double c[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) c[s] = y[s] > 0.0 ? y[s] / M::W[s] : 0.0;
  double T = T_from_e<M>(c, rho, e, *Tio);
  const double h = dt / nsub;
  for (int sub = 0; sub < nsub; sub++) {
    const double lnT = log(T), invT = 1.0 / T;
    const double lnP0RT = log(PATM / (RU * T));
    double g[NS];
    {
      // below TLO the constant-cp extrapolation of mechanism.hpp mech_gibbs,
      // branch-free: at Te = max(T, TLO) the polynomial terms, then with
      // r = Te / T and dl = lnT - lnTe
      //   g = hRT(Te) r + cp/R (1 - r) - s/R(Te) - cp/R dl,
      // which for T >= TLO (r = 1, dl = 0; no contraction) is hRT - s/R bit
      // for bit.  (A branch to a separate low-T loop cost this kernel 50
      // registers and 18 % of its time.)
      const bool lo = T < TLO;
      const double Te = lo ? TLO : T, lnTe = lo ? log(TLO) : lnT;
      const double r = lo ? TLO * invT : 1.0, dl = lnT - lnTe;
#pragma unroll
      for (int s = 0; s < NS; s++) {
        const double* a = coef<M>(s, Te);
        const double hRT = a[0] + Te * (a[1] * 0.5 + Te * (a[2] * (1.0 / 3.0) + Te * (a[3] * 0.25 + Te * a[4] * 0.2))) +
                           a[5] / Te;
        const double sR = a[0] * lnTe + Te * (a[1] + Te * (a[2] * 0.5 + Te * (a[3] * (1.0 / 3.0) + Te * a[4] * 0.25))) + a[6];
        const double cpR = a[0] + Te * (a[1] + Te * (a[2] + Te * (a[3] + Te * a[4])));
        g[s] = hRT * r + cpR * (1.0 - r) - sR - cpR * dl;
      }
    }
    constexpr int NA = Reacting<M>::N;
    constexpr auto X = Reacting<M>::map;
    double A[NA][NA + 1];
#pragma unroll
    for (int i = 0; i < NA; i++)
#pragma unroll
      for (int j = 0; j <= NA; j++) A[i][j] = (i == j) ? 1.0 : 0.0;
    apply_all<M>(MakeSeq<M::NR>{}, c, g, T, lnT, invT, lnP0RT, h, A);
    if (!solve<NA>(A)) break;
    double tot = 0.0;
#pragma unroll
    for (int s = 0; s < NS; s++) {
      c[s] = c[s] + (X.ix[s] >= 0 ? A[X.ix[s] >= 0 ? X.ix[s] : 0][NA] : 0.0);
      c[s] = c[s] < 0.0 ? 0.0 : c[s];
      tot += c[s] * M::W[s];
    }
    const double sc = tot > 0.0 ? rho / tot : 1.0;
#pragma unroll
    for (int s = 0; s < NS; s++) c[s] *= sc;
    T = T_from_e<M>(c, rho, e, T);
  }
#pragma unroll
  for (int s = 0; s < NS; s++) y[s] = c[s] * M::W[s];
  *Tio = T;
}


// ---- kernel bodies (one cell per lane, 256-lane workgroups) ----
template <class M>
__device__ void chem_dense_body(const ChemArgs& a) {
  const double dt = args_dt(a);
  const long idx = a.c0 + (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= a.c1) return;
  constexpr int NS = M::NS;
  const long N = a.N;
  double y[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) y[s] = a.Yin[(long)s * N + idx];
  const double rho = a.S[idx];
  const double T0 = a.Tprev[idx];
  if (args_active(a, a.CT[idx]) && rho > 0.0 && T0 >= a.Tchem && dt > 0.0) {
    const double ru = a.S[(long)1 * N + idx], rv = a.S[(long)2 * N + idx];
    const double e = (a.S[(long)3 * N + idx] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
    double T = T0;
    chem_cell<M>(rho, e, y, &T, dt, a.nsub);
  }
#pragma unroll
  for (int s = 0; s < NS; s++) a.Yout[(long)s * N + idx] = y[s];
}

// Compacted form.  On the scramjet only 2-5 % of the cells are above Tchem,
// but 16-20 % of the 64-cell wavefronts hold at least one of them, and a
// wavefront costs as much as its slowest lane.  Pass 1 copies the species of
// every cell that stays frozen and appends the reacting cells to a list
// (one atomic per wavefront); pass 2 integrates the listed cells densely.
// Cells are independent, so the result does not depend on the list order.
template <class M>
__device__ void chem_mark_body(const ChemArgs& a) {
  const double dt = args_dt(a);
  const long idx = a.c0 + (long)blockIdx.x * 256 + threadIdx.x;
  const bool in = idx < a.c1;
  const bool hot = in && args_active(a, a.CT[idx]) && a.S[idx] > 0.0 && a.Tprev[idx] >= a.Tchem && dt > 0.0;
  const long N = a.N;
  if (in && !hot) {
#pragma unroll
    for (int s = 0; s < M::NS; s++) a.Yout[(long)s * N + idx] = a.Yin[(long)s * N + idx];
  }
  const unsigned long long ball = __ballot(hot);
  if (!ball) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)ball) - 1;
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(a.count, (unsigned)__popcll(ball));
  base = __shfl(base, leader, 64);
  if (hot) a.list[base + __popcll(ball & ((1ull << lane) - 1ull))] = (int)idx;
}

template <class M>
__device__ void chem_list_body(const ChemArgs& a) {
  const double dt = args_dt(a);
  const unsigned n = *a.count;
  constexpr int NS = M::NS;
  const long N = a.N;
  for (unsigned k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const long idx = a.list[k];
    double y[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) y[s] = a.Yin[(long)s * N + idx];
    const double rho = a.S[idx];
    const double ru = a.S[(long)1 * N + idx], rv = a.S[(long)2 * N + idx];
    const double e = (a.S[(long)3 * N + idx] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
    double T = a.Tprev[idx];
    chem_cell<M>(rho, e, y, &T, dt, a.nsub);
#pragma unroll
    for (int s = 0; s < NS; s++) a.Yout[(long)s * N + idx] = y[s];
  }
}

// standalone operator (tests / benchmarks): rhoY [ns][n] in place at (rho, e)
template <class M>
__device__ void chem_op_body(double* rhoY, const double* rho, const double* e, double* T, long n, double dt, int nsub) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  double y[M::NS];
#pragma unroll
  for (int s = 0; s < M::NS; s++) y[s] = rhoY[(long)s * n + q];
  double Tq = T[q];
  chem_cell<M>(rho[q], e[q], y, &Tq, dt, nsub);
#pragma unroll
  for (int s = 0; s < M::NS; s++) rhoY[(long)s * n + q] = y[s];
  T[q] = Tq;
}

}  // namespace chemk
}  // namespace hf2d
