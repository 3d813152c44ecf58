#include <algorithm>
// K12 (mechanism mode): operator-split kinetics with a compiled mechanism,
// one cell per lane, everything in registers (gfx950, FP64).  The
// integrator and kernel bodies are chem_fast_dev.hpp (shared with the
// hiprtc-compiled kernels of file mechanisms, chem_rtc.hip); this unit
// instantiates them for the built-in mechanisms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "chem_fast.hpp"
#include "chem_fast_dev.hpp"
#include "dev_common.hpp"
#include "mech_h2_air_li2004.hpp"

namespace hf2d {
namespace {

using chemk::ChemArgs;

// (the integrating kernels at a 2-wave register budget, as hf2d_chem_fast_list)
template <class M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void hf2d_chem_fast(ChemArgs a) {
  chemk::chem_dense_body<M>(a);
}
template <class M>
__global__ __launch_bounds__(256) void hf2d_chem_fast_mark(ChemArgs a) {
  chemk::chem_mark_body<M>(a);
}
// (a 2-wave register budget: 256 VGPRs with 42 spilled (116 B scratch)
// instead of 286 registers at one wave per SIMD; the developed scramjet
// state's kinetics 0.202 -> 0.165 ms per step, profiles/scramjet_phases_r05.log)
template <class M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void hf2d_chem_fast_list(ChemArgs a) {
  chemk::chem_list_body<M>(a);
}
template <class M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void hf2d_chem_fast_op(double* rhoY, const double* rho, const double* e, double* T,
                                                         long n, double dt, int nsub) {
  chemk::chem_op_body<M>(rhoY, rho, e, T, n, dt, nsub);
}

}  // namespace

// (FP32 build, HF2D_FP32: the kinetics kernels work on FP64 state only; the
// mechanism mode is not available there)
#ifdef HF2D_FP32
bool chem_fast_available(const std::string&) { return false; }
#else
bool chem_fast_available(const std::string& mech) { return mech == "h2_air_li2004"; }
#endif

ChemArgs chem_args(const SoA& mid, const SoA& out, const real* Tprev, long c0, long c1, DevScalars* sc, int slot,
                   double Tchem, int nsub, int* list, unsigned* count) {
  ChemArgs a;
#ifdef HF2D_FP32
  (void)mid, (void)out, (void)Tprev, (void)c0, (void)c1, (void)sc, (void)slot, (void)Tchem, (void)nsub, (void)list,
      (void)count;
  throw std::runtime_error("FP32 build: the finite-rate kinetics kernels need the FP64 build");
#else
  a.S = mid.S;
  a.Yin = mid.Ys;
  a.Yout = out.Ys;
  a.Tprev = Tprev;
  a.CT = (const unsigned long long*)mid.CT;   // u64 is unsigned long: same width
  a.dt_bits = &sc->dt_bits[slot];
  a.N = mid.N;
  a.c0 = c0;
  a.c1 = c1;
  a.Tchem = Tchem;
  a.nsub = nsub;
  a.set_bit = CT_NODE_IS_SET;
  a.solid_bit = CT_SOLID;
  a.fc_bits = NT_FC;
  a.list = list;
  a.count = count;
#endif
  return a;
}

bool chem_fast_launch(const std::string& mech, const StepParams& P, const SoA& mid, const SoA& out, const real* Tprev,
                      long c0, long c1, DevScalars* sc, int slot, double Tchem, int nsub, hipStream_t st, int* list,
                      unsigned* count, bool list_ready) {
  (void)P;
  if (mech != "h2_air_li2004" || mid.nsp != Mech_h2_air_li2004::NS) return false;
  const unsigned nb = (unsigned)((c1 - c0 + 255) / 256);
  if (nb == 0) return true;
  const ChemArgs a = chem_args(mid, out, Tprev, c0, c1, sc, slot, Tchem, nsub, list, count);
  // (grid-stride over the list; 4096 workgroups measured best in the developed
  // scramjet state: kinetics 0.166 ms vs 0.172 / 0.173 ms at 1024 / 512)
  if (list && count && list_ready) {
    hipLaunchKernelGGL(hf2d_chem_fast_list<Mech_h2_air_li2004>, dim3(std::min(nb, 4096u)), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess;
  }
  if (list && count) {   // compacted: frozen cells copied, reacting cells integrated densely
    if (hipMemsetAsync(count, 0, sizeof(unsigned), st) != hipSuccess) return false;
    hipLaunchKernelGGL(hf2d_chem_fast_mark<Mech_h2_air_li2004>, dim3(nb), dim3(256), 0, st, a);
    // grid-stride over the list: enough workgroups for a fully reacting grid
    // to fill the chip several times, without knowing the count on the host
    const unsigned gl = std::min(nb, 4096u);
    hipLaunchKernelGGL(hf2d_chem_fast_list<Mech_h2_air_li2004>, dim3(gl), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess;
  }
  hipLaunchKernelGGL(hf2d_chem_fast<Mech_h2_air_li2004>, dim3(nb), dim3(256), 0, st, a);
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
