#include <algorithm>
// K12 (mechanism mode): operator-split kinetics with a compiled mechanism,
// one cell per lane, everything in registers (gfx950, FP64).
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
// template parameter (tools/gen_mech_header.py): every reaction is a separate
// instantiation (index_sequence), all species indices are compile-time
// constants, the 9x10 system of a cell lives in VGPRs and only the non-zero
// Jacobian entries are accumulated.  Runtime (file) mechanisms use the MFMA
// kernel.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <utility>

#include "chem_fast.hpp"
#include "dev_common.hpp"
#include "mech_h2_air_li2004.hpp"

namespace hf2d {
namespace {

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
template <class M>
__device__ __forceinline__ void mix_e_cv(const double* c, double rho, double T, double* e, double* cv) {
  double se = 0.0, scv = 0.0;
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
  *e = se * MECH_RU / rho;
  *cv = scv * MECH_RU / rho;
}

template <class M>
__device__ double T_from_e(const double* c, double rho, double e, double T0) {
  double T = T0 > MECH_TMIN ? (T0 < MECH_TMAX ? T0 : MECH_TMAX) : MECH_TMIN;
  for (int it = 0; it < 30; it++) {
    double ee, cv;
    mix_e_cv<M>(c, rho, T, &ee, &cv);
    double dT = (e - ee) / cv;
    dT = dT > 500.0 ? 500.0 : (dT < -500.0 ? -500.0 : dT);
    double Tn = T + dT;
    Tn = Tn > MECH_TMIN ? (Tn < MECH_TMAX ? Tn : MECH_TMAX) : MECH_TMIN;
    const double d = Tn - T;
    T = Tn;
    if (fabs(d) <= 1e-10 * T) break;
  }
  return T;
}

// One reaction's contribution to the augmented system A = [I - h J | h w].
template <class M, int R>
__device__ __forceinline__ void apply_rx(const double* c, const double* g, double T, double lnT, double invT,
                                         double lnP0RT, double h, double (&A)[M::NS][M::NS + 1]) {
  constexpr CRx r = M::rx[R];
  constexpr int NS = M::NS;
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
  for (int t = 0; t < r.nrs; t++) A[r.rs[t]][NS] -= r.rn[t] * hq;
#pragma unroll
  for (int t = 0; t < r.nps; t++) A[r.ps[t]][NS] += r.pn[t] * hq;
  // -h nu_i D_j, D_j = dq/dc_j
  auto put = [&](int j, double Dj) {
#pragma unroll
    for (int t = 0; t < r.nrs; t++) A[r.rs[t]][j] += r.rn[t] * h * Dj;
#pragma unroll
    for (int t = 0; t < r.nps; t++) A[r.ps[t]][j] -= r.pn[t] * h * Dj;
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
__device__ __forceinline__ void apply_all(std::integer_sequence<int, Rs...>, const double* c, const double* g, double T,
                                          double lnT, double invT, double lnP0RT, double h,
                                          double (&A)[M::NS][M::NS + 1]) {
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
    const double lnP0RT = log(MECH_PATM / (MECH_RU * T));
    double g[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const double* a = coef<M>(s, T);
      const double hRT = a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2))) +
                         a[5] / T;
      const double sR = a[0] * lnT + T * (a[1] + T * (a[2] * 0.5 + T * (a[3] * (1.0 / 3.0) + T * a[4] * 0.25))) + a[6];
      g[s] = hRT - sR;
    }
    double A[NS][NS + 1];
#pragma unroll
    for (int i = 0; i < NS; i++)
#pragma unroll
      for (int j = 0; j <= NS; j++) A[i][j] = (i == j) ? 1.0 : 0.0;
    apply_all<M>(std::make_integer_sequence<int, M::NR>{}, c, g, T, lnT, invT, lnP0RT, h, A);
    if (!solve<NS>(A)) break;
    double tot = 0.0;
#pragma unroll
    for (int s = 0; s < NS; s++) {
      c[s] = c[s] + A[s][NS];
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

template <class M>
__global__ __launch_bounds__(256) void hf2d_chem_fast(StepParams P, SoA mid, SoA out, const real* Tprev, long c0,
                                                      long c1, DevScalars* sc, int slot, double Tchem, int nsub) {
  apply_dt(P, sc, slot);
  const long idx = c0 + (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= c1) return;
  constexpr int NS = M::NS;
  const long N = mid.N;
  double y[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) y[s] = mid.Ys[(long)s * N + idx];
  const double rho = mid.S[idx];
  const double T0 = Tprev[idx];
  if (is_active(mid.CT[idx]) && rho > 0.0 && T0 >= Tchem && P.dt > 0.0) {
    const double ru = mid.S[(long)I_RHOU * N + idx], rv = mid.S[(long)I_RHOV * N + idx];
    const double e = (mid.S[(long)I_RHOE * N + idx] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
    double T = T0;
    chem_cell<M>(rho, e, y, &T, P.dt, nsub);
  }
#pragma unroll
  for (int s = 0; s < NS; s++) out.Ys[(long)s * N + idx] = y[s];
}

// Compacted form.  On the scramjet only 2-5 % of the cells are above Tchem,
// but 16-20 % of the 64-cell wavefronts hold at least one of them, and a
// wavefront costs as much as its slowest lane.  Pass 1 copies the species of
// every cell that stays frozen and appends the reacting cells to a list
// (one atomic per wavefront); pass 2 integrates the listed cells densely.
// Cells are independent, so the result does not depend on the list order.
__device__ inline bool chem_hot(const StepParams& P, const SoA& mid, const real* Tprev, long idx, double Tchem) {
  return is_active(mid.CT[idx]) && mid.S[idx] > 0.0 && Tprev[idx] >= Tchem && P.dt > 0.0;
}

template <class M>
__global__ __launch_bounds__(256) void hf2d_chem_fast_mark(StepParams P, SoA mid, SoA out, const real* Tprev, long c0,
                                                           long c1, DevScalars* sc, int slot, double Tchem,
                                                           int* list, unsigned* count) {
  apply_dt(P, sc, slot);
  const long idx = c0 + (long)blockIdx.x * 256 + threadIdx.x;
  const bool in = idx < c1;
  const bool hot = in && chem_hot(P, mid, Tprev, idx, Tchem);
  const long N = mid.N;
  if (in && !hot) {
#pragma unroll
    for (int s = 0; s < M::NS; s++) out.Ys[(long)s * N + idx] = mid.Ys[(long)s * N + idx];
  }
  const unsigned long long ball = __ballot(hot);
  if (!ball) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)ball) - 1;
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(count, (unsigned)__popcll(ball));
  base = __shfl(base, leader, 64);
  if (hot) list[base + __popcll(ball & ((1ull << lane) - 1ull))] = (int)idx;
}

template <class M>
__global__ __launch_bounds__(256) void hf2d_chem_fast_list(StepParams P, SoA mid, SoA out, const real* Tprev,
                                                           DevScalars* sc, int slot, int nsub, const int* list,
                                                           const unsigned* count) {
  apply_dt(P, sc, slot);
  const unsigned n = *count;
  constexpr int NS = M::NS;
  const long N = mid.N;
  for (unsigned k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const long idx = list[k];
    double y[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) y[s] = mid.Ys[(long)s * N + idx];
    const double rho = mid.S[idx];
    const double ru = mid.S[(long)I_RHOU * N + idx], rv = mid.S[(long)I_RHOV * N + idx];
    const double e = (mid.S[(long)I_RHOE * N + idx] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
    double T = Tprev[idx];
    chem_cell<M>(rho, e, y, &T, P.dt, nsub);
#pragma unroll
    for (int s = 0; s < NS; s++) out.Ys[(long)s * N + idx] = y[s];
  }
}

// standalone operator (tests / benchmarks): rhoY [ns][n] in place at (rho, e)
template <class M>
__global__ __launch_bounds__(256) void hf2d_chem_fast_op(double* rhoY, const double* rho, const double* e, double* T,
                                                         long n, double dt, int nsub) {
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

}  // namespace

bool chem_fast_available(const std::string& mech) { return mech == "h2_air_li2004"; }

bool chem_fast_launch(const std::string& mech, const StepParams& P, const SoA& mid, const SoA& out, const real* Tprev,
                      long c0, long c1, DevScalars* sc, int slot, double Tchem, int nsub, hipStream_t st, int* list,
                      unsigned* count) {
  if (mech != "h2_air_li2004" || mid.nsp != Mech_h2_air_li2004::NS) return false;
  const unsigned nb = (unsigned)((c1 - c0 + 255) / 256);
  if (nb == 0) return true;
  if (list && count) {   // compacted: frozen cells copied, reacting cells integrated densely
    if (hipMemsetAsync(count, 0, sizeof(unsigned), st) != hipSuccess) return false;
    hipLaunchKernelGGL(hf2d_chem_fast_mark<Mech_h2_air_li2004>, dim3(nb), dim3(256), 0, st, P, mid, out, Tprev, c0, c1,
                       sc, slot, Tchem, list, count);
    // grid-stride over the list: enough workgroups for a fully reacting grid
    // to fill the chip several times, without knowing the count on the host
    const unsigned gl = std::min(nb, 4096u);
    hipLaunchKernelGGL(hf2d_chem_fast_list<Mech_h2_air_li2004>, dim3(gl), dim3(256), 0, st, P, mid, out, Tprev, sc,
                       slot, nsub, list, count);
    return hipGetLastError() == hipSuccess;
  }
  hipLaunchKernelGGL(hf2d_chem_fast<Mech_h2_air_li2004>, dim3(nb), dim3(256), 0, st, P, mid, out, Tprev, c0, c1, sc,
                     slot, Tchem, nsub);
  return hipGetLastError() == hipSuccess;
}

double chem_fast_run_host(const std::string& mech, double* rhoY, const double* rho, const double* e, double* T, long n,
                          double dt, int nsub, int repeats) {
  if (mech != "h2_air_li2004") throw std::runtime_error("chem_fast: no compiled kernel for " + mech);
  constexpr int NS = Mech_h2_air_li2004::NS;
  struct Buf {
    void* p = nullptr;
    ~Buf() {
      if (p) (void)hipFree(p);
    }
  } dY, dY0, drho, de, dT, dT0;
  auto ck = [](hipError_t r, const char* w) {
    if (r != hipSuccess) throw std::runtime_error(std::string("chem_fast: ") + w + ": " + hipGetErrorString(r));
  };
  const size_t nb = sizeof(double) * n;
  ck(hipMalloc(&dY.p, nb * NS), "malloc");
  ck(hipMalloc(&dY0.p, nb * NS), "malloc");
  ck(hipMalloc(&drho.p, nb), "malloc");
  ck(hipMalloc(&de.p, nb), "malloc");
  ck(hipMalloc(&dT.p, nb), "malloc");
  ck(hipMalloc(&dT0.p, nb), "malloc");
  ck(hipMemcpy(dY0.p, rhoY, nb * NS, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(drho.p, rho, nb, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(de.p, e, nb, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(dT0.p, T, nb, hipMemcpyHostToDevice), "h2d");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ck(hipEventCreate(&e0), "event");
  ck(hipEventCreate(&e1), "event");
  float total = 0.f;
  const unsigned g = (unsigned)((n + 255) / 256);
  for (int it = 0; it < (repeats > 0 ? repeats : 1); it++) {
    ck(hipMemcpy(dY.p, dY0.p, nb * NS, hipMemcpyDeviceToDevice), "d2d");
    ck(hipMemcpy(dT.p, dT0.p, nb, hipMemcpyDeviceToDevice), "d2d");
    ck(hipEventRecord(e0, 0), "record");
    hipLaunchKernelGGL(hf2d_chem_fast_op<Mech_h2_air_li2004>, dim3(g), dim3(256), 0, 0, (double*)dY.p,
                       (const double*)drho.p, (const double*)de.p, (double*)dT.p, n, dt, nsub);
    ck(hipGetLastError(), "launch");
    ck(hipEventRecord(e1, 0), "record");
    ck(hipEventSynchronize(e1), "sync");
    float ms = 0.f;
    ck(hipEventElapsedTime(&ms, e0, e1), "elapsed");
    total += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  ck(hipMemcpy(rhoY, dY.p, nb * NS, hipMemcpyDeviceToHost), "d2h");
  ck(hipMemcpy(T, dT.p, nb, hipMemcpyDeviceToHost), "d2h");
  return total / (repeats > 0 ? repeats : 1);
}

}  // namespace hf2d
