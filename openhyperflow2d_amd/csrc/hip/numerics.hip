// Device numerics probe: hf_div / hf_sqrt (core/common.hpp) evaluated on the
// GPU for host-supplied operands, so tests can check them bit for bit
// against IEEE division / square root (numpy) -- the claim the lean kernels'
// CPU == GPU bitwise equality rests on.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "core/common.hpp"
#include "hip/numerics.hpp"

namespace hf2d {

__global__ void hf2d_div_probe(const double* a, const double* b, double* q, double* s, long n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  q[t] = hf_div(a[t], b[t]);
  s[t] = hf_sqrt(a[t]);
}

void div_probe(const double* a, const double* b, double* q, double* s, long n) {
  if (n <= 0) return;
  double* d = nullptr;
  auto ck = [](hipError_t e, const char* w) {
    if (e != hipSuccess) throw std::runtime_error(std::string("div_probe: ") + w + ": " + hipGetErrorString(e));
  };
  ck(hipMalloc((void**)&d, 4 * n * sizeof(double)), "hipMalloc");
  ck(hipMemcpy(d, a, n * sizeof(double), hipMemcpyHostToDevice), "copy a");
  ck(hipMemcpy(d + n, b, n * sizeof(double), hipMemcpyHostToDevice), "copy b");
  const unsigned nb = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(hf2d_div_probe, dim3(nb), dim3(256), 0, 0, d, d + n, d + 2 * n, d + 3 * n, n);
  ck(hipGetLastError(), "launch");
  ck(hipMemcpy(q, d + 2 * n, n * sizeof(double), hipMemcpyDeviceToHost), "copy q");
  ck(hipMemcpy(s, d + 3 * n, n * sizeof(double), hipMemcpyDeviceToHost), "copy s");
  ck(hipFree(d), "hipFree");
}

}  // namespace hf2d
