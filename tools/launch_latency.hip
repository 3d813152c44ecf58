// Host <-> GPU round trip of one small kernel launch + stream synchronize,
// under each hipSetDeviceFlags scheduling mode (set before any other HIP
// call, in a child process per mode):
//   hipcc --offload-arch=gfx950 -O2 tools/launch_latency.hip -o tools/launch_latency
//   tools/launch_latency            (spawns itself once per mode)
//   tools/launch_latency <mode>     (0 auto, 1 spin, 2 yield, 4 blocking sync)
// Prints the median / p10 of 2000 round trips, and of chains of 20 kernels
// of ~25 us each (the headline bench's call shape).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// ~us of busy work per workgroup (s_memrealtime: 100 MHz)
__global__ void busy(int* p, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && blockIdx.x == 0) p[1] += 1;
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

static int run(int mode) {
  if (hipSetDeviceFlags((unsigned)mode) != hipSuccess) std::printf("mode %d: hipSetDeviceFlags failed\n", mode);
  int* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  (void)hipMemset(d, 0, 64);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int k = 0; k < 100; k++) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
  (void)hipStreamSynchronize(s);
  std::vector<double> one, chain;
  for (int k = 0; k < 2000; k++) {
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    one.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
  }
  for (int k = 0; k < 200; k++) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int q = 0; q < 20; q++) hipLaunchKernelGGL(busy, dim3(1024), dim3(256), 0, s, d, 2500ull);
    (void)hipStreamSynchronize(s);
    chain.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
  }
  std::printf("{\"mode\": %d, \"launch_sync_us_p50\": %.2f, \"p10\": %.2f, \"chain20x25us_p50\": %.2f, \"p10_chain\": %.2f}\n",
              mode, pct(one, 0.5), pct(one, 0.1), pct(chain, 0.5), pct(chain, 0.1));
  (void)hipFree(d);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1) return run(std::atoi(argv[1]));
  int rc = 0;
  for (int mode : {0, 1, 2, 4}) {
    const std::string cmd = std::string(argv[0]) + " " + std::to_string(mode);
    rc |= std::system(cmd.c_str());   // a fresh process per mode (the flags bind at context creation)
  }
  return rc;
}
