// K12: finite-rate multi-reaction chemistry on the MFMA matrix cores (gfx950, FP64).
//
// The reference has only the "infinite speed" Zeldovich global reaction
// (deeps2d_core.cpp:4697-4780) and an empty CRM_ARRENIUS slot
// (hyper_flow_bound.hpp:37-42); SURVEY.md 2.4 K12 asks for a finite-rate kinetics
// kernel with per-cell Jacobians on MFMA.  This kernel advances a mass-action
// mechanism (ns <= 16 species, R reactions, R % 4 == 0, irreversible Arrhenius
// steps with integer reactant orders; a reversible step is two entries) by
// nsub linearised backward-Euler (point-implicit) substeps at frozen T:
//
//     (I - h J) dc = h N q(c),   J = N D,   D[r][j] = dq_r / dc_j,   c <- max(c + dc, 0)
//
// with c = rhoY / W [mol/m^3] and N = nu'' - nu' (ns x R).  Both matrix products
// are MFMA work (v_mfma_f64_16x16x4_f64, one wavefront = one 16-cell tile):
//   * rates   Omega(16 species x 16 cells) = N(16 x R) . Q(R x 16 cells)   R/4 MFMAs
//   * Jacobian J_c(16 x 16)                = N(16 x R) . D_c(R x 16)       R/4 MFMAs per cell
// and the 16x16 systems are solved by Gauss-Jordan with partial pivoting, 16 lanes
// per cell (lane = row, held in registers), 4 cells at a time, staged through LDS.
// The 4 Jacobians of a round are independent MFMA chains (latency hiding).
//
// f64 MFMA operand maps (cdna_hip_programming.md): A[row=l&15][k=l>>4],
// B[k=l>>4][col=l&15], C/D col=l&15, row=(l>>4)+4*i.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "chem_mech.hpp"

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int TILE = 16;     // cells per wavefront (MFMA N dimension)
constexpr int MAXR = 64;     // reactions per mechanism
constexpr int LD = 18;       // row stride of the staged systems (16 cols + rhs + pad)

// x^o for o in 0..3 without branches
__device__ __forceinline__ double pw3(double x, int o) {
  const double x2 = x * x;
  return o == 0 ? 1.0 : (o == 1 ? x : (o == 2 ? x2 : x2 * x));
}

// NSP: system size (ns rounded up to a multiple of 4).  Rows/columns >= ns carry an
// identity block (no reaction touches them), so only the NSP x NSP block and the rhs
// are eliminated.
template <int NSP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void hf2d_chem_mech(const double* __restrict__ nmat,   // [16][R]
                                                     const double* __restrict__ arr,    // A[R], b[R], Ta[R]
                                                     const int* __restrict__ rsp,       // [R][3]
                                                     const int* __restrict__ rord,      // [R][3]
                                                     const double* __restrict__ W,      // [ns]
                                                     int ns, int R, int ncell, double* __restrict__ rhoY,
                                                     const double* __restrict__ T, double dt, int nsub) {
  __shared__ double c_s[TILE][TILE + 1];        // [cell][species]
  __shared__ double m_s[4][TILE][LD];           // 4 systems in flight: [cell][row][col | rhs]
  __shared__ double x_s[4][TILE];
  __shared__ int rx_s[MAXR];                    // packed reactants: 3 x (species 4 bits, order 2 bits)
  extern __shared__ double kf_dyn[];            // [cell][R + 1] rate constants (sized per mechanism)

  const int l = threadIdx.x, col = l & 15, quad = l >> 4;
  const int cell0 = blockIdx.x * TILE;
  const int mycell = cell0 + col;
  const bool live = mycell < ncell;

  for (int r = l; r < R; r += 64) {
    int pk = 0;
    for (int t = 0; t < 3; t++) pk |= (rsp[r * 3 + t] | (rord[r * 3 + t] << 4)) << (6 * t);
    rx_s[r] = pk;
  }
  for (int i = 0; i < 4; i++) {
    const int s = quad + 4 * i;
    c_s[col][s] = (live && s < ns) ? rhoY[(size_t)s * ncell + mycell] / W[s] : 0.0;
  }
  {
    const double Tc = live ? T[mycell] : 300.0;
    const double lnT = log(Tc), rT = 1.0 / Tc;
    for (int r = quad; r < R; r += 4) kf_dyn[col * (R + 1) + r] = arr[r] * exp(arr[R + r] * lnT - arr[2 * R + r] * rT);
  }
  const double h = dt / nsub;

  for (int sub = 0; sub < nsub; sub++) {
    __syncthreads();
    // Omega[s][cell] = sum_r N[s][r] q[r][cell]; lane (quad, col): Omega[quad + 4 i][col]
    d4 om = {0.0, 0.0, 0.0, 0.0};
    for (int r0 = 0; r0 < R; r0 += 4) {
      const int r = r0 + quad, pk = rx_s[r];
      double q = kf_dyn[col * (R + 1) + r];
#pragma unroll
      for (int t = 0; t < 3; t++) q *= pw3(c_s[col][(pk >> (6 * t)) & 15], (pk >> (6 * t + 4)) & 3);
      om = __builtin_amdgcn_mfma_f64_16x16x4f64(nmat[col * R + r], q, om, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; g++) {
      // Jacobians of cells 4g..4g+3 as 4 independent MFMA chains:
      // J_cc = N D_cc, B operand D_cc[r = r0 + quad][j = col].
      d4 jac[4];
#pragma unroll
      for (int qq = 0; qq < 4; qq++) jac[qq] = d4{0.0, 0.0, 0.0, 0.0};
      for (int r0 = 0; r0 < R; r0 += 4) {
        const int r = r0 + quad, pk = rx_s[r];
        const double nv = nmat[col * R + r];
        const int s0 = pk & 15, o0 = (pk >> 4) & 3, s1 = (pk >> 6) & 15, o1 = (pk >> 10) & 3, s2 = (pk >> 12) & 15,
                  o2 = (pk >> 16) & 3;
        const bool h0 = s0 == col && o0 > 0, h1 = s1 == col && o1 > 0, h2 = s2 == col && o2 > 0;
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
          const int cc = 4 * g + qq;
          const double c0 = c_s[cc][s0], c1 = c_s[cc][s1], c2 = c_s[cc][s2];
          const double p0 = pw3(c0, o0), p1 = pw3(c1, o1), p2 = pw3(c2, o2);
          const double kf = kf_dyn[cc * (R + 1) + r];
          double d = 0.0;
          if (h0) d = kf * (o0 * pw3(c0, o0 - 1)) * p1 * p2;
          if (h1) d = kf * p0 * (o1 * pw3(c1, o1 - 1)) * p2;
          if (h2) d = kf * p0 * p1 * (o2 * pw3(c2, o2 - 1));
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
      __syncthreads();
      double row[TILE + 1];
#pragma unroll
      for (int j = 0; j <= TILE; j++) row[j] = m_s[quad][col][j];

      // Gauss-Jordan, group `quad` solves cell 4g+quad; lane `col` holds row col in
      // registers (k, j unrolled), the pivot row is read with in-group shuffles.
      bool used = false;
      int kk = 0;
      double diag = 1.0;
#pragma unroll
      for (int k = 0; k < NSP; k++) {
        // Pivot = max |M[i][k]| over unused rows, ties to the lower row: one 64-bit key per
        // lane (|v|'s bits, monotone for v >= 0, low 4 mantissa bits replaced by 15 - row).
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
        const double f = me ? 0.0 : row[k] / pk;
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
      if (used) x_s[quad][kk] = row[TILE] / diag;
      __syncthreads();
      {
        const int cc = 4 * g + quad;
        if (col < ns) c_s[cc][col] = fmax(c_s[cc][col] + x_s[quad][col], 0.0);
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (live)
    for (int i = 0; i < 4; i++) {
      const int s = quad + 4 * i;
      if (s < ns) rhoY[(size_t)s * ncell + mycell] = c_s[col][s] * W[s];
    }
}

}  // namespace

namespace hf2d {

int chem_mech_max_reactions() { return MAXR; }

// Device pointers; returns a hipError_t code (0 = ok).
int chem_mech_launch(const ChemMechDev& m, double* rhoY, const double* T, int ncell, double dt, int nsub,
                     hipStream_t stream) {
  if (m.ns < 1 || m.ns > TILE || m.R < 4 || m.R % 4 != 0 || m.R > MAXR || ncell < 1 || nsub < 1)
    return (int)hipErrorInvalidValue;
  const int blocks = (ncell + TILE - 1) / TILE;
  const size_t lds = sizeof(double) * TILE * (m.R + 1);
#define HF2D_CHEM_LAUNCH(N)                                                                                  \
  hipLaunchKernelGGL(hf2d_chem_mech<N>, dim3(blocks), dim3(64), lds, stream, m.nmat, m.arr, m.rsp, m.rord, m.W, \
                     m.ns, m.R, ncell, rhoY, T, dt, nsub)
  switch ((m.ns + 3) / 4) {
    case 1: HF2D_CHEM_LAUNCH(4); break;
    case 2: HF2D_CHEM_LAUNCH(8); break;
    case 3: HF2D_CHEM_LAUNCH(12); break;
    default: HF2D_CHEM_LAUNCH(16); break;
  }
#undef HF2D_CHEM_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace hf2d

namespace hf2d {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("chem_mech: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

double chem_mech_run_host(const double* nmat, const double* arr, const int* rsp, const int* rord, const double* W,
                          int ns, int R, double* rhoY, const double* T, int ncell, double dt, int nsub,
                          int repeats) {
  if (ns < 1 || ns > 16 || R < 4 || R % 4 != 0 || R > MAXR || ncell < 1 || nsub < 1)
    throw std::runtime_error("chem_mech: need 1 <= ns <= 16, 4 <= R <= 64 with R % 4 == 0, ncell >= 1, nsub >= 1");
  for (int i = 0; i < 3 * R; i++)
    if (rsp[i] < 0 || rsp[i] >= ns || rord[i] < 0 || rord[i] > 3)
      throw std::runtime_error("chem_mech: reactant species out of range or order not in 0..3");
  const size_t nY = (size_t)ns * ncell;
  double *d_nmat, *d_arr, *d_W, *d_Y, *d_Y0, *d_T;
  int *d_rsp, *d_rord;
  ck(hipMalloc(&d_nmat, sizeof(double) * 16 * R), "malloc");
  ck(hipMalloc(&d_arr, sizeof(double) * 3 * R), "malloc");
  ck(hipMalloc(&d_W, sizeof(double) * ns), "malloc");
  ck(hipMalloc(&d_rsp, sizeof(int) * 3 * R), "malloc");
  ck(hipMalloc(&d_rord, sizeof(int) * 3 * R), "malloc");
  ck(hipMalloc(&d_Y, sizeof(double) * nY), "malloc");
  ck(hipMalloc(&d_Y0, sizeof(double) * nY), "malloc");
  ck(hipMalloc(&d_T, sizeof(double) * ncell), "malloc");
  ck(hipMemcpy(d_nmat, nmat, sizeof(double) * 16 * R, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_arr, arr, sizeof(double) * 3 * R, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_W, W, sizeof(double) * ns, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_rsp, rsp, sizeof(int) * 3 * R, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_rord, rord, sizeof(int) * 3 * R, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_Y0, rhoY, sizeof(double) * nY, hipMemcpyHostToDevice), "h2d");
  ck(hipMemcpy(d_T, T, sizeof(double) * ncell, hipMemcpyHostToDevice), "h2d");
  ChemMechDev m;
  m.nmat = d_nmat; m.arr = d_arr; m.rsp = d_rsp; m.rord = d_rord; m.W = d_W; m.ns = ns; m.R = R;
  hipEvent_t e0, e1;
  ck(hipEventCreate(&e0), "event");
  ck(hipEventCreate(&e1), "event");
  float total = 0.f;
  for (int it = 0; it < std::max(repeats, 1); it++) {
    ck(hipMemcpyAsync(d_Y, d_Y0, sizeof(double) * nY, hipMemcpyDeviceToDevice, 0), "d2d");
    ck(hipEventRecord(e0, 0), "record");
    ck((hipError_t)chem_mech_launch(m, d_Y, d_T, ncell, dt, nsub, 0), "launch");
    ck(hipEventRecord(e1, 0), "record");
    ck(hipEventSynchronize(e1), "sync");
    float ms = 0.f;
    ck(hipEventElapsedTime(&ms, e0, e1), "elapsed");
    total += ms;
  }
  ck(hipMemcpy(rhoY, d_Y, sizeof(double) * nY, hipMemcpyDeviceToHost), "d2h");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  for (void* p : {(void*)d_nmat, (void*)d_arr, (void*)d_W, (void*)d_rsp, (void*)d_rord, (void*)d_Y, (void*)d_Y0,
                  (void*)d_T})
    (void)hipFree(p);
  return total / std::max(repeats, 1);
}

}  // namespace hf2d
