// K12 for runtime (file) mechanisms on the MFMA matrix cores (gfx950, FP64).
//
// Mechanism mode's kinetics operator (core/mechanism.hpp mech_chem_cell is the
// host oracle; chem_fast.hip the register-resident kernel for compiled
// mechanisms): nsub linearised backward-Euler substeps (I - h J) dc = h w at
// constant rho and e with reversible rates, third-body efficiencies, Troe
// fall-off and T re-solved from e after every substep.  A mechanism loaded at
// run time has no compile-time structure, so the reaction-space algebra is
// done as dense 16x16 tiles on the matrix cores, one wavefront = 16 cells
// (the MFMA N dimension), v_mfma_f64_16x16x4_f64 throughout:
//   ln Kc (R x cells) = -N^T (R x 16 sp) . G (16 sp x cells)      Gibbs energies
//   [M]   (R x cells) =  E   (R x 16 sp) . C (16 sp x cells)      collider conc.
//   w     (16 sp x cells) = N (16 x R) . Q (R x cells)            net rates
//   J_c   (16 x 16) = N (16 x R) . D_c (R x 16)  per cell          Jacobian
// Per-(cell, reaction) scalars (k_f, fall-off, k_r = k_f / Kc, q, dq/dc) run
// in the MFMA output layout; the 16x16 systems are solved by Gauss-Jordan
// with partial pivoting, 16 lanes per cell, 4 cells at a time, staged
// through LDS.
//
// f64 MFMA operand maps (cdna_hip_programming.md): A[row=l&15][k=l>>4],
// B[k=l>>4][col=l&15], C/D col=l&15, row=(l>>4)+4*i.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../core/mechanism.hpp"
#include "chem_mech.hpp"

namespace hf2d {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int TILE = 16;     // cells per wavefront (MFMA N dimension)
constexpr int MAXR = 64;     // reactions per mechanism (multiple of 16 after padding)
constexpr int LD = 18;       // row stride of the staged systems (16 cols + rhs + pad)

__device__ __forceinline__ double pw3(double x, int o) {
  const double x2 = x * x;
  return o == 0 ? 1.0 : (o == 1 ? x : (o == 2 ? x2 : x2 * x));
}

__device__ __forceinline__ const double* nasa(const ChemMechDev& m, int s, double T) {
  return m.thermo + (s * 2 + (T < m.thermo[16 * 14 + s] ? 0 : 1)) * 7;
}

// specific internal energy and cv of the concentrations of one cell at T
// (below MECH_TLO: constant-cp extrapolation, as mech_mix_thermo)
__device__ void cell_e_cv(const ChemMechDev& m, const double* c, double rho, double Tin, double* e, double* cv) {
  double se = 0.0, scv = 0.0;
  const double T = Tin < MECH_TLO ? MECH_TLO : Tin;
  for (int s = 0; s < m.ns; s++) {
    const double* a = nasa(m, s, T);
    const double cpR = a[0] + T * (a[1] + T * (a[2] + T * (a[3] + T * a[4])));
    const double hRT = a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2))) + a[5] / T;
    se += c[s] * (T * (hRT - 1.0));
    scv += c[s] * (cpR - 1.0);
  }
  se += scv * (Tin - T);   // (+0 for Tin >= MECH_TLO)
  *e = se * MECH_RU / rho;
  *cv = scv * MECH_RU / rho;
}

__device__ double cell_T(const ChemMechDev& m, const double* c, double rho, double e, double T0) {
  double T = T0 > MECH_TMIN ? (T0 < MECH_TMAX ? T0 : MECH_TMAX) : MECH_TMIN;
  for (int it = 0; it < 30; it++) {
    double ee, cv;
    cell_e_cv(m, c, rho, T, &ee, &cv);
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

// NSP: system size (ns rounded up to 4); rows/columns >= ns are identity.
template <int NSP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void hf2d_chem_mech(
    ChemMechDev m, MechCells q, double dt, int nsub) {
  __shared__ double c_s[TILE][TILE + 1];        // [cell][species] concentrations
  __shared__ double g_s[TILE][TILE + 1];        // [cell][species] Gibbs h/RT - s/R
  __shared__ double m_s[4][TILE][LD];           // 4 systems in flight: [cell][row][col | rhs]
  __shared__ double x_s[4][TILE];
  __shared__ double cellv[4][TILE];             // rho, e, T, lnP0RT per cell
  __shared__ int rx_s[MAXR], px_s[MAXR], fl_s[MAXR];
  extern __shared__ double dyn[];               // kf | kr | mult: [3][cell][R + 1]

  const int l = threadIdx.x, col = l & 15, quad = l >> 4;
  const int R = m.R;
  if (q.dt_bits) dt = __longlong_as_double((long long)*q.dt_bits);
  double* kf_d = dyn;
  double* kr_d = dyn + TILE * (R + 1);
  double* mu_d = dyn + 2 * TILE * (R + 1);
  const long cell = q.c0 + (long)blockIdx.x * TILE + col;
  bool live = cell < q.c1;
  // only active, warm cells react; the rest of the tile computes on a dummy
  // state (T = 1000 K, c = 1) and does not store
  bool react = false;
  if (live) {
    const double rho = q.S[cell];
    react = q.active(cell) && rho > 0 && q.Tprev[cell] >= q.Tchem && dt > 0;
  }
  for (int r = l; r < R; r += 64) {
    rx_s[r] = m.rx[r * 4 + 0];
    px_s[r] = m.rx[r * 4 + 1];
    fl_s[r] = m.rx[r * 4 + 2];
  }
  for (int i = 0; i < 4; i++) {
    const int s = quad + 4 * i;
    double v = 0.0;
    if (s < m.ns) v = react ? fmax(q.Yin[(long)s * q.N + cell], 0.0) / m.W[s] : 1.0;
    c_s[col][s] = v;
  }
  if (quad == 0) {
    double rho = 1.0, e = 0.0, T = 1000.0;
    if (react) {
      rho = q.S[cell];
      const double ru = q.S[(long)I_RHOU * q.N + cell], rv = q.S[(long)I_RHOV * q.N + cell];
      e = (q.S[(long)I_RHOE * q.N + cell] - 0.5 * (ru * ru + rv * rv) / rho) / rho;
      T = q.Tprev[cell];
    }
    cellv[0][col] = rho;
    cellv[1][col] = e;
    cellv[2][col] = T;
  }
  __syncthreads();
  if (quad == 0) {
    double c[TILE];
    for (int s = 0; s < TILE; s++) c[s] = c_s[col][s];
    if (react) cellv[2][col] = cell_T(m, c, cellv[0][col], cellv[1][col], cellv[2][col]);
  }
  const double h = dt / nsub;

  for (int sub = 0; sub < nsub; sub++) {
    __syncthreads();
    // --- per-cell thermodynamics: Gibbs energies of every species ---------
    {
      const double T = cellv[2][col], lnT = log(T);
      for (int i = 0; i < 4; i++) {
        const int s = quad + 4 * i;
        double gv = 0.0;
        if (s < m.ns && T < MECH_TLO) {   // constant-cp extrapolation (mechanism.hpp mech_gibbs)
          const double Te = MECH_TLO, lnTe = log(MECH_TLO);
          const double* a = nasa(m, s, Te);
          const double cpR = a[0] + Te * (a[1] + Te * (a[2] + Te * (a[3] + Te * a[4])));
          const double hT =
              Te * (a[0] + Te * (a[1] * 0.5 + Te * (a[2] * (1.0 / 3.0) + Te * (a[3] * 0.25 + Te * a[4] * 0.2)))) + a[5];
          const double sR =
              a[0] * lnTe + Te * (a[1] + Te * (a[2] * 0.5 + Te * (a[3] * (1.0 / 3.0) + Te * a[4] * 0.25))) + a[6];
          gv = (hT + cpR * (T - Te)) / T - (sR + cpR * (lnT - lnTe));
        } else if (s < m.ns) {
          const double* a = nasa(m, s, T);
          const double hRT =
              a[0] + T * (a[1] * 0.5 + T * (a[2] * (1.0 / 3.0) + T * (a[3] * 0.25 + T * a[4] * 0.2))) + a[5] / T;
          const double sR = a[0] * lnT + T * (a[1] + T * (a[2] * 0.5 + T * (a[3] * (1.0 / 3.0) + T * a[4] * 0.25))) + a[6];
          gv = hRT - sR;
        }
        g_s[col][s] = gv;
      }
      if (quad == 0) cellv[3][col] = log(MECH_PATM / (MECH_RU * T));
    }
    __syncthreads();
    // --- rate constants: ln Kc and [M] as MFMA tiles, scalars in the D layout --
    for (int rt = 0; rt < R; rt += 16) {
      d4 lk = {0.0, 0.0, 0.0, 0.0}, mm = {0.0, 0.0, 0.0, 0.0};
      for (int ks = 0; ks < NSP; ks += 4) {
        const int s = ks + quad, r = rt + col;
        const double an = -m.nmat[s * R + r];            // A[row r][k s]
        const double ae = m.eff[r * 16 + s];
        lk = __builtin_amdgcn_mfma_f64_16x16x4f64(an, g_s[col][s], lk, 0, 0, 0);   // B[k s][col cell]
        mm = __builtin_amdgcn_mfma_f64_16x16x4f64(ae, c_s[col][s], mm, 0, 0, 0);
      }
      const double T = cellv[2][col], lnT = log(T), invT = 1.0 / T, lp = cellv[3][col];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = rt + quad + 4 * i;   // D row; column = cell `col`
        const int fl = fl_s[r];
        double kf = m.arr[r] * exp(m.arr[R + r] * lnT - m.arr[2 * R + r] * invT);
        double mult = 1.0;
        if (fl & 4) {   // fall-off
          const double k0 = m.fall[r] * exp(m.fall[R + r] * lnT - m.fall[2 * R + r] * invT);
          const double Pr = k0 * mm[i] / kf;
          double F = 1.0;
          const int nt = (fl >> 3) & 7;
          if (nt >= 3) {
            const double a = m.fall[3 * R + r];
            double Fc = (1.0 - a) * exp(-T / m.fall[4 * R + r]) + a * exp(-T / m.fall[5 * R + r]);
            if (nt > 3) Fc += exp(-m.fall[6 * R + r] * invT);
            const double lFc = log10(Fc > 1e-300 ? Fc : 1e-300);
            const double lPr = log10(Pr > 1e-300 ? Pr : 1e-300);
            const double cc = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;
            const double f1 = (lPr + cc) / (nn - 0.14 * (lPr + cc));
            F = pow(10.0, lFc / (1.0 + f1 * f1));
          }
          kf = kf * (Pr / (1.0 + Pr)) * F;
        } else if (fl & 2) {   // "+ M"
          mult = mm[i];
        }
        const int dnu = (fl >> 8) - 16;
        const double kr = (fl & 1) ? kf * exp(-(lk[i] + dnu * lp)) : 0.0;
        kf_d[col * (R + 1) + r] = kf;
        kr_d[col * (R + 1) + r] = kr;
        mu_d[col * (R + 1) + r] = mult;
      }
    }
    __syncthreads();
    // --- net rates w = N . Q ------------------------------------------------
    d4 om = {0.0, 0.0, 0.0, 0.0};
    for (int r0 = 0; r0 < R; r0 += 4) {
      const int r = r0 + quad, pk = rx_s[r], pp = px_s[r];
      double pf = kf_d[col * (R + 1) + r], pr = kr_d[col * (R + 1) + r];
#pragma unroll
      for (int t = 0; t < 3; t++) {
        pf *= pw3(c_s[col][(pk >> (6 * t)) & 15], (pk >> (6 * t + 4)) & 3);
        pr *= pw3(c_s[col][(pp >> (6 * t)) & 15], (pp >> (6 * t + 4)) & 3);
      }
      om = __builtin_amdgcn_mfma_f64_16x16x4f64(m.nmat[col * R + r], mu_d[col * (R + 1) + r] * (pf - pr), om, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; g++) {
      // Jacobians of cells 4g..4g+3 as 4 independent MFMA chains:
      // J_cc = N D_cc, B operand D_cc[r = r0 + quad][j = col].
      d4 jac[4];
#pragma unroll
      for (int qq = 0; qq < 4; qq++) jac[qq] = d4{0.0, 0.0, 0.0, 0.0};
      for (int r0 = 0; r0 < R; r0 += 4) {
        const int r = r0 + quad, pk = rx_s[r], pp = px_s[r], fl = fl_s[r];
        const double nv = m.nmat[col * R + r];
        const double ev = ((fl & 6) == 2) ? m.eff[r * 16 + col] : 0.0;   // pure third body
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
          const int cc = 4 * g + qq;
          const double kf = kf_d[cc * (R + 1) + r], kr = kr_d[cc * (R + 1) + r], mu = mu_d[cc * (R + 1) + r];
          double pf = kf, pr = kr, df = 0.0, dr = 0.0;
#pragma unroll
          for (int t = 0; t < 3; t++) {
            const int sf = (pk >> (6 * t)) & 15, of = (pk >> (6 * t + 4)) & 3;
            const int sr = (pp >> (6 * t)) & 15, orr = (pp >> (6 * t + 4)) & 3;
            const double cf = c_s[cc][sf], cr = c_s[cc][sr];
            // d(prod)/dc_col by the product rule over the (distinct) species
            df = df * pw3(cf, of) + ((sf == col && of > 0) ? pf * (of * pw3(cf, of - 1)) : 0.0);
            dr = dr * pw3(cr, orr) + ((sr == col && orr > 0) ? pr * (orr * pw3(cr, orr - 1)) : 0.0);
            pf *= pw3(cf, of);
            pr *= pw3(cr, orr);
          }
          const double d = mu * (df - dr) + ev * (pf - pr);
          jac[qq] = __builtin_amdgcn_mfma_f64_16x16x4f64(nv, d, jac[qq], 0, 0, 0);
        }
      }
#pragma unroll
      for (int qq = 0; qq < 4; qq++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int s = quad + 4 * i;
          m_s[qq][s][col] = (s == col ? 1.0 : 0.0) - h * jac[qq][i];
        }
      if ((col >> 2) == g)
        for (int i = 0; i < 4; i++) m_s[col & 3][quad + 4 * i][TILE] = h * om[i];
      x_s[quad][col] = 0.0;
      __syncthreads();
      double row[TILE + 1];
#pragma unroll
      for (int j = 0; j <= TILE; j++) row[j] = m_s[quad][col][j];

      // Gauss-Jordan, group `quad` solves cell 4g+quad; lane `col` holds row col
      bool used = false;
      int kk = 0;
      double diag = 1.0;
#pragma unroll
      for (int k = 0; k < NSP; k++) {
        // pivot = max |M[i][k]| over unused rows (ties to the lower row): one
        // 64-bit key per lane, |v|'s bits with the low 4 replaced by 15 - row
        unsigned long long key =
            used ? 0ull : ((unsigned long long)__double_as_longlong(fabs(row[k])) & ~15ull) | (unsigned)(15 - col);
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          const unsigned long long ok = __shfl_xor(key, off, 16);
          key = ok > key ? ok : key;
        }
        const int p = 15 - (int)(key & 15ull);
        const double pk = __shfl(row[k], p, 16);
        const bool me = col == p;
        const double f = (me || pk == 0.0) ? 0.0 : row[k] / pk;
        if (me) {
          used = true;
          kk = k;
          diag = row[k];
        } else {
          row[k] = 0.0;
        }
#pragma unroll
        for (int j = k + 1; j <= TILE; j++)
          if (j < NSP || j == TILE) row[j] -= f * __shfl(row[j], p, 16);
      }
      // a singular system (zero pivot) leaves that cell's species unchanged
      if (used && kk < m.ns) x_s[quad][kk] = fabs(diag) > 0.0 ? row[TILE] / diag : 0.0;
      __syncthreads();
      {
        const int cc = 4 * g + quad;
        if (col < m.ns) c_s[cc][col] = fmax(c_s[cc][col] + x_s[quad][col], 0.0);
      }
      __syncthreads();
    }
    // mass re-normalisation and T from e, one lane per cell
    if (quad == 0) {
      double c[TILE], tot = 0.0;
      for (int s = 0; s < TILE; s++) {
        c[s] = c_s[col][s];
        if (s < m.ns) tot += c[s] * m.W[s];
      }
      const double rho = cellv[0][col];
      const double sc = tot > 0.0 ? rho / tot : 1.0;
      for (int s = 0; s < m.ns; s++) {
        c[s] *= sc;
        c_s[col][s] = c[s];
      }
      if (react) cellv[2][col] = cell_T(m, c, rho, cellv[1][col], cellv[2][col]);
    }
  }
  __syncthreads();
  if (live) {
    for (int i = 0; i < 4; i++) {
      const int s = quad + 4 * i;
      if (s < m.ns) q.Yout[(long)s * q.N + cell] = react ? c_s[col][s] * m.W[s] : q.Yin[(long)s * q.N + cell];
    }
    if (quad == 0 && q.Tout) q.Tout[cell] = react ? cellv[2][col] : q.Tprev[cell];
  }
}

}  // namespace

int chem_mech_max_reactions() { return MAXR; }

int chem_mech_launch(const ChemMechDev& m, const MechCells& q, double dt, int nsub, hipStream_t stream) {
  if (m.ns < 1 || m.ns > TILE || m.R < 16 || m.R % 16 != 0 || m.R > MAXR || nsub < 1) return (int)hipErrorInvalidValue;
  if (q.c1 <= q.c0) return 0;
  const unsigned blocks = (unsigned)((q.c1 - q.c0 + TILE - 1) / TILE);
  const size_t lds = sizeof(double) * 3 * TILE * (m.R + 1);
#define HF2D_CHEM_LAUNCH(N) \
  hipLaunchKernelGGL(hf2d_chem_mech<N>, dim3(blocks), dim3(64), lds, stream, m, q, dt, nsub)
  switch ((m.ns + 3) / 4) {
    case 1: HF2D_CHEM_LAUNCH(4); break;
    case 2: HF2D_CHEM_LAUNCH(8); break;
    case 3: HF2D_CHEM_LAUNCH(12); break;
    default: HF2D_CHEM_LAUNCH(16); break;
  }
#undef HF2D_CHEM_LAUNCH
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Device pack of a MechData (owned device buffers)
// ---------------------------------------------------------------------------
namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("chem_mech: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

ChemMechPack::~ChemMechPack() {
  for (void* p : bufs) (void)hipFree(p);
}

std::unique_ptr<ChemMechPack> chem_mech_pack(const MechData& md) {
  std::unique_ptr<ChemMechPack> pk(new ChemMechPack);
  const int R = std::max(16, (md.nr + 15) / 16 * 16);
  if (md.ns > 16 || R > MAXR) throw std::runtime_error("chem_mech: at most 16 species and 64 reactions");
  std::vector<double> nmat(16 * R, 0.0), arr(3 * R, 0.0), fall(7 * R, 0.0), eff(R * 16, 0.0);
  std::vector<double> thermo(16 * 14 + 16 + 16, 0.0);
  std::vector<int> rx(R * 4, 0);
  for (int s = 0; s < md.ns; s++) {
    for (int b = 0; b < 2; b++)
      for (int k = 0; k < 7; k++) thermo[(s * 2 + b) * 7 + k] = md.a[s][b][k];
    thermo[16 * 14 + s] = md.Tmid[s];
  }
  for (int s = md.ns; s < 16; s++) thermo[16 * 14 + s] = 1000.0;
  for (int r = 0; r < R; r++) {
    int fl = 16 << 8;   // dnu = 0
    if (r < md.nr) {
      const MechReaction& x = md.rx[r];
      int pr = 0, pp = 0;
      for (int t = 0; t < x.nrs; t++) {
        nmat[x.rs[t] * R + r] -= x.rn[t];
        pr |= (x.rs[t] | (x.rn[t] << 4)) << (6 * t);
      }
      for (int t = 0; t < x.nps; t++) {
        nmat[x.ps[t] * R + r] += x.pn[t];
        pp |= (x.ps[t] | (x.pn[t] << 4)) << (6 * t);
      }
      arr[r] = x.A;
      arr[R + r] = x.b;
      arr[2 * R + r] = x.Ta;
      fall[r] = x.A0;
      fall[R + r] = x.b0;
      fall[2 * R + r] = x.Ta0;
      for (int k = 0; k < 4; k++) fall[(3 + k) * R + r] = x.troe[k];
      if (x.tb || x.fo)
        for (int s = 0; s < md.ns; s++) eff[r * 16 + s] = x.eff >= 0 ? md.eff[x.eff][s] : 1.0;
      fl = (x.rev ? 1 : 0) | ((x.tb && !x.fo) ? 2 : 0) | (x.fo ? 4 : 0) | ((x.ntroe & 7) << 3) | ((x.dnu + 16) << 8);
      rx[r * 4 + 0] = pr;
      rx[r * 4 + 1] = pp;
    } else {
      arr[r] = 0.0;   // padding reaction: k = 0
    }
    rx[r * 4 + 2] = fl;
  }
  auto up = [&](const void* h, size_t bytes) {
    void* d = nullptr;
    ck(hipMalloc(&d, std::max<size_t>(bytes, 8)), "malloc");
    pk->bufs.push_back(d);
    ck(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice), "h2d");
    return d;
  };
  std::vector<double> W(16, 1.0);
  for (int s = 0; s < md.ns; s++) W[s] = md.W[s];
  ChemMechDev& m = pk->dev;
  m.nmat = (const double*)up(nmat.data(), nmat.size() * 8);
  m.arr = (const double*)up(arr.data(), arr.size() * 8);
  m.fall = (const double*)up(fall.data(), fall.size() * 8);
  m.eff = (const double*)up(eff.data(), eff.size() * 8);
  m.thermo = (const double*)up(thermo.data(), thermo.size() * 8);
  m.W = (const double*)up(W.data(), W.size() * 8);
  m.rx = (const int*)up(rx.data(), rx.size() * 4);
  m.ns = md.ns;
  m.R = R;
  return pk;
}

// Runtime-data VALU form of the operator: one cell per lane, the host
// integrator's template (core/mechanism.hpp mech_chem_cell) over the
// MechData block in device memory.  Like hf2d_chem_mech, and unlike the
// compiled chem_fast / hiprtc kernels, every stoichiometric coefficient, rate
// parameter and efficiency is read at run time, so the two measure the
// matrix cores against the vector ALUs on the same work.
__global__ __launch_bounds__(64) void hf2d_chem_rt_valu(const MechData* md, MechCells q, double dt, int nsub) {
  const long cell = q.c0 + (long)blockIdx.x * 64 + threadIdx.x;
  if (cell >= q.c1) return;
  const int ns = md->ns;
  double rhoY[MECH_MAXSP];
  for (int s = 0; s < ns; s++) rhoY[s] = q.Yin[(long)s * q.N + cell];
  const double rho = q.S[cell];
  const double e = q.S[3 * q.N + cell] / rho;   // (at rest: the standalone operator's states)
  double T = q.Tprev[cell];
#ifndef HF2D_FP32   // (FP32 build: the FP64 kinetics of this comparison kernel are not compiled)
  mech_chem_cell<MECH_MAXSP>(*md, rho, e, rhoY, &T, dt, nsub);
#endif
  for (int s = 0; s < ns; s++) q.Yout[(long)s * q.N + cell] = rhoY[s];
  q.Tout[cell] = T;
}

double chem_mech_run_host(const MechData& md, double* rhoY, const double* rho, const double* e, double* T, long n,
                          double dt, int nsub, int repeats, bool valu) {
  if (n < 1 || nsub < 1) throw std::runtime_error("chem_mech: need n >= 1 and nsub >= 1");
  for (long i = 0; i < n; i++)
    if (!(T[i] > 0.0) || !(rho[i] > 0.0)) throw std::runtime_error("chem_mech: T and rho must be > 0 and finite");
  auto pk = chem_mech_pack(md);
  const int ns = md.ns;
  // the solver's SoA form: S = [rho, rhoU = 0, rhoV = 0, rho*e], every cell active
  std::vector<double> S(4 * n), Y((size_t)ns * n);
  for (long i = 0; i < n; i++) {
    S[i] = rho[i];
    S[n + i] = S[2 * n + i] = 0.0;
    S[3 * n + i] = rho[i] * e[i];
  }
  struct Buf {
    void* p = nullptr;
    ~Buf() {
      if (p) (void)hipFree(p);
    }
  } dS, dY0, dY, dT0, dT;
  const size_t nb = sizeof(double) * n;
  ck(hipMalloc(&dS.p, 4 * nb), "malloc");
  ck(hipMalloc(&dY0.p, ns * nb), "malloc");
  ck(hipMalloc(&dY.p, ns * nb), "malloc");
  ck(hipMalloc(&dT0.p, nb), "malloc");
  ck(hipMalloc(&dT.p, nb), "malloc");
  ck(hipMemcpy(dS.p, S.data(), 4 * nb, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(dY0.p, rhoY, ns * nb, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(dT0.p, T, nb, hipMemcpyHostToDevice), "h2d");
  MechCells q;
  q.S = (const double*)dS.p;
  q.Yin = (const double*)dY0.p;
  q.Yout = (double*)dY.p;
  q.Tprev = (const double*)dT0.p;
  q.Tout = (double*)dT.p;
  q.CT = nullptr;
  q.N = n;
  q.c0 = 0;
  q.c1 = n;
  q.Tchem = 0.0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ck(hipEventCreate(&e0), "event");
  ck(hipEventCreate(&e1), "event");
  float total = 0.f;
  struct DevMech {
    MechData* p = nullptr;
    ~DevMech() {
      if (p) (void)hipFree(p);
    }
  } dm;
  if (valu) {
    ck(hipMalloc(&dm.p, sizeof(MechData)), "malloc");
    ck(hipMemcpy(dm.p, &md, sizeof(MechData), hipMemcpyHostToDevice), "h2d");
  }
  for (int it = 0; it < std::max(repeats, 1); it++) {
    ck(hipEventRecord(e0, 0), "record");
    if (valu) {
      hipLaunchKernelGGL(hf2d_chem_rt_valu, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, dm.p, q, dt, nsub);
      ck(hipGetLastError(), "launch");
    } else {
      ck((hipError_t)chem_mech_launch(pk->dev, q, dt, nsub, 0), "launch");
    }
    ck(hipEventRecord(e1, 0), "record");
    ck(hipEventSynchronize(e1), "sync");
    float ms = 0.f;
    ck(hipEventElapsedTime(&ms, e0, e1), "elapsed");
    total += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  ck(hipMemcpy(rhoY, dY.p, ns * nb, hipMemcpyDeviceToHost), "d2h");
  ck(hipMemcpy(T, dT.p, nb, hipMemcpyDeviceToHost), "d2h");
  return total / std::max(repeats, 1);
}

}  // namespace hf2d
