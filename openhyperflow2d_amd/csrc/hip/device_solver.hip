// GPU backend for MI355X (gfx950): device-resident SoA state, one HIP
// kernel per DEEPS phase, RCCL halo exchange / reductions for strip-
// decomposed multi-GPU runs.
//
// Kernels (rocprof names):
//   hf2d_predict<RES>     pass 1 + 2a (predictor, BC, residual, blending factor)
//   hf2d_fill             pass 2b/2c (gradients, FillNode2D, dt, chemistry)
//   hf2d_fused_euler      predict + fill in one sweep for Euler problems
//   hf2d_lean_euler       inviscid step on the reduced state (lean_euler.hpp):
//                         fluxes recomputed from neighbour state, ~1/5 the
//                         HBM traffic of predict+fill
//   hf2d_lean_materialize rebuild A/B/F/p from the lean state
//   hf2d_wall_solid/_wall owner-computes wall heat sources (K5)
//   hf2d_reduce_residual  deterministic tree over per-wave residual partials (K6)
//   hf2d_pack/unpack      halo column packing (K7)
//   hf2d_yplus            per-cycle y+ (K10)
// dt never leaves the device inside the inner loop: hf2d_fill folds the
// local CFL limit into a device slot with an integer atomicMin on the IEEE
// bits (valid for positive doubles, order independent => deterministic) and
// the next step's kernels read it from there.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../core/lean_euler.hpp"
#include "../core/solver.hpp"
#include "device_solver.hpp"
#include "dev_common.hpp"
#include "chem_fast.hpp"
#include "chem_rtc.hpp"
#include "chem_mech.hpp"
#include "lean_ns.hpp"
#include "lean_mech.hpp"

#define HIP_CHECK(x)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess)                                                                        \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " +      \
                               __FILE__ + ":" + std::to_string(__LINE__));                       \
  } while (0)
#define NCCL_CHECK(x)                                                                            \
  do {                                                                                           \
    ncclResult_t r_ = (x);                                                                       \
    if (r_ != ncclSuccess)                                                                       \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r_) + " at " +    \
                               __FILE__ + ":" + std::to_string(__LINE__));                       \
  } while (0)

namespace hf2d {

constexpr int BLOCK = 256;
constexpr int WAVE = 64;

// ---------------------------------------------------------------------------
// Wave-level residual reduction helpers
// ---------------------------------------------------------------------------
__device__ inline void shfl_merge(ResidualPack& r, int off) {
#pragma unroll
  for (int k = 0; k < NEQ; k++) {
    EqResidual o;
    o.dd_max = __shfl_xor(r.eq[k].dd_max, off, WAVE);
    o.i = __shfl_xor(r.eq[k].i, off, WAVE);
    o.j = __shfl_xor(r.eq[k].j, off, WAVE);
    o.rms = __shfl_xor(r.eq[k].rms, off, WAVE);
    o.sum_div = __shfl_xor(r.eq[k].sum_div, off, WAVE);
    o.count = __shfl_xor(r.eq[k].count, off, WAVE);
    EqResidual& f = r.eq[k];
    const bool later = (o.i > f.i) || (o.i == f.i && o.j > f.j);
    if (o.dd_max > f.dd_max || (o.dd_max == f.dd_max && later)) {
      f.dd_max = o.dd_max;
      f.i = o.i;
      f.j = o.j;
    }
    f.rms += o.rms;
    f.sum_div += o.sum_div;
    f.count += o.count;
  }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2).  Remap so XCD x owns a contiguous run of tiles: the i+-1 neighbour
// columns a tile reads then sit in the same L2.  Bijective on [0, n).
constexpr unsigned NUM_XCD = 8;
__device__ inline unsigned xcd_remap(unsigned b, unsigned n) {
  const unsigned q = n / NUM_XCD;
  if (b >= q * NUM_XCD) return b;
  return (b % NUM_XCD) * q + b / NUM_XCD;
}
// Split kernels (one cell per thread, x-major): logical block of this
// workgroup.  A column of a tall grid spans a few blocks, so the left/right
// neighbour reads of the round-robin order land on another XCD's L2; with
// StepParams::xcd the blocks of an XCD form one contiguous column range.
__device__ inline unsigned split_block(const StepParams& P) {
  return P.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
}

template <bool RES, int MODE = SK_GENERIC>
__global__ __launch_bounds__(BLOCK) void hf2d_predict(StepParams P, SoA in, SoA out, long c0, long c1,
                                                       DevScalars* sc, int slot, int slot_next, int serial,
                                                       ResidualPack* partials) {
  apply_dt(P, sc, slot);
  const unsigned blk = split_block(P);
  const long g = (long)blk * BLOCK + threadIdx.x;
  if (g == 0) {
    // Reset the slot the NEXT step will accumulate into (never the one this
    // step's fill is min-reducing, which other blocks may already be
    // writing) and accumulate physical time.
    dt_reset(sc, slot_reset(slot));
    lag_head(P, sc, slot, slot_next);
    sc->dt_bits[slot] = d_to_bits(P.dt);   // folded (later kernels of the step read the word)
    sc->time_part += P.dt;
    sc->dt_val[slot] = P.dt;
    sc->hot_cnt[slot_next] = 0;
    scenario_next(P, sc, slot, slot_next);
  }
  const long c = c0 + g;
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  if (c < c1) {
    const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
    predict_cell_t<RES, MODE>(P, in, out, i, j, r);
  }
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)blk * (BLOCK / WAVE) + threadIdx.x / WAVE] = r;
  }
}

__global__ __launch_bounds__(BLOCK) void hf2d_reduce_residual(const ResidualPack* partials, long n,
                                                               ResidualPack* outp) {
  __shared__ ResidualPack sh[32];
  ResidualPack acc;
  residual_reset(acc);
  for (int k = 0; k < NEQ; k++) acc.eq[k].i = acc.eq[k].j = -1;
  for (long t = threadIdx.x; t < n; t += BLOCK) residual_merge_lex(acc, partials[t]);
  for (int off = 1; off < WAVE; off <<= 1) shfl_merge(acc, off);
  const int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    ResidualPack a = sh[0];
    for (int q = 1; q < BLOCK / WAVE; q++) residual_merge_lex(a, sh[q]);
    *outp = a;
  }
}

template <int MODE, int NSB, bool LAZY = false>
__device__ __forceinline__ void fill_body(StepParams& P, const SoA& sin, const SoA& pold, const SoA& out, long c0,
                                          long c1, DevScalars* sc, int slot, int slot_next, int serial,
                                          int store_grad);

template <int MODE = SK_GENERIC, int NSB = 1>
__global__ __launch_bounds__(BLOCK) void hf2d_fill(StepParams P, SoA sin, SoA pold, SoA out, long c0, long c1,
                                                    DevScalars* sc, int slot, int slot_next, int serial,
                                                    int store_grad) {
  fill_body<MODE, NSB>(P, sin, pold, out, c0, c1, sc, slot, slot_next, serial, store_grad);
}

// The same fill with a register budget of OCC waves per SIMD (the split N-S
// fills compile to 165-255 VGPRs, i.e. 1-3 waves; DeviceSolver::fill_occ)
template <int MODE, int NSB, int OCC, bool LAZY = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(OCC))) void hf2d_fill_occ(
    StepParams P, SoA sin, SoA pold, SoA out, long c0, long c1, DevScalars* sc, int slot, int slot_next, int serial,
    int store_grad) {
  fill_body<MODE, NSB, LAZY>(P, sin, pold, out, c0, c1, sc, slot, slot_next, serial, store_grad);
}

template <int MODE, int NSB, bool LAZY>
__device__ __forceinline__ void fill_body(StepParams& P, const SoA& sin, const SoA& pold, const SoA& out, long c0,
                                          long c1, DevScalars* sc, int slot, int slot_next, int serial,
                                          int store_grad) {
  apply_dt(P, sc, slot);
  const long c = c0 + (long)split_block(P) * BLOCK + threadIdx.x;
  double dtl = 1.0;
  int neg = 0;
  if (c < c1) {
    const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
    dtl = fill_cell<MODE, NSB, LAZY>(P, sin, pold, out, i, j, &neg, store_grad != 0);
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) m = fmin(m, sdt[q]);
    if (serial) m = fmin(m, P.dt);  // serial build: dt is a running minimum
    if (slot_next >= 0) dt_min(sc, slot_next, m);   // < 0: lean N-S materialize
  }
}

// Mechanism mode, operator-split kinetics (runtime mechanism data; the
// per-cell point-implicit integrator of mechanism.hpp): predicted species
// mid.Ys -> out.Ys over the step's dt at constant rho and e.
template <int NSB>
__global__ __launch_bounds__(BLOCK) void hf2d_chem_generic(StepParams P, SoA mid, SoA out, const real* Tprev, long c0,
                                                            long c1, DevScalars* sc, int slot) {
  apply_dt(P, sc, slot);
  const long c = c0 + (long)blockIdx.x * BLOCK + threadIdx.x;
  if (c < c1) {
    const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
    mech_chem_soa_cell<NSB>(P, mid, out, Tprev, i, j);
  }
}

// Euler: no gradients, so the fill of a cell depends only on its own
// predicted state and the predictor and fill run in one sweep.  A and B are
// ping-ponged (neighbours read the old fluxes).
template <bool RES>
__global__ __launch_bounds__(BLOCK) void hf2d_fused_euler(StepParams P, SoA in, SoA mid, SoA out, long c0, long c1,
                                                           DevScalars* sc, int slot, int slot_next, int serial,
                                                           ResidualPack* partials) {
  apply_dt(P, sc, slot);
  const long g = (long)blockIdx.x * BLOCK + threadIdx.x;
  if (g == 0) {
    dt_reset(sc, slot_reset(slot));
    lag_head(P, sc, slot, slot_next);
    sc->dt_bits[slot] = d_to_bits(P.dt);   // folded (later kernels of the step read the word)
    sc->time_part += P.dt;
    scenario_next(P, sc, slot, slot_next);
  }
  const long c = c0 + g;
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  double dtl = 1.0;
  int neg = 0;
  if (c < c1) {
    const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
    predict_cell_t<RES>(P, in, mid, i, j, r);
    dtl = fill_cell(P, mid, mid, out, i, j, &neg, false);
  }
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)blockIdx.x * (BLOCK / WAVE) + threadIdx.x / WAVE] = r;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) m = fmin(m, sdt[q]);
    if (serial) m = fmin(m, P.dt);  // serial build: dt is a running minimum
    if (slot_next >= 0) dt_min(sc, slot_next, m);   // < 0: lean N-S materialize
  }
}

template <bool RES, bool FROMG>
__global__ __launch_bounds__(BLOCK) void hf2d_lean_euler(StepParams P, LeanSoA L, long c0, long c1, DevScalars* sc,
                                                          int slot, int slot_next, int serial,
                                                          ResidualPack* partials) {
  apply_dt(P, sc, slot);
  const unsigned b = xcd_remap(blockIdx.x, gridDim.x);
  const long g = (long)b * BLOCK + threadIdx.x;
  if (g == 0) {
    dt_reset(sc, slot_reset(slot));
    lag_head(P, sc, slot, slot_next);
    sc->dt_bits[slot] = d_to_bits(P.dt);   // folded (later kernels of the step read the word)
    sc->time_part += P.dt;
    scenario_next(P, sc, slot, slot_next);
  }
  const long c = c0 + g;
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  double dtl = 1.0;
  int neg = 0;
  if (c < c1) {
    const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
    dtl = lean_euler_cell<RES, FROMG>(P, L, i, j, r, &neg);
  }
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)b * (BLOCK / WAVE) + threadIdx.x / WAVE] = r;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) m = fmin(m, sdt[q]);
    if (serial) m = fmin(m, P.dt);
    dt_min(sc, slot_next, m);
  }
}

// Halo pack: nf field columns (each ny contiguous doubles at src[f] + col*ny)
constexpr int MAX_HALO_FIELDS = 128;   // 4*NEQ + 5 state fields + up to 16 species x 4
// Halo field list: entry f is column (first + o[f]) / (last - o[f]) of
// field f on the sending side and ghost column (ghostL - o[f]) / (ghostR +
// o[f]) on the receiving side: o = 1 carries the second column of a
// two-column halo (the lean N-S / mechanism kernels on strips).
struct ColList {
  real* f[MAX_HALO_FIELDS];
  unsigned char o[MAX_HALO_FIELDS] = {};
  int nf;
};
constexpr long P2P_SPIN_LIMIT = 1L << 26;   // ~3 s of s_sleep polling, then give up (neg_T bit 2)
constexpr int P2P_THREADS = 512;

// Acquire load of a peer's publication flag at system scope: the poll loops
// spin with relaxed loads (cheap) and finish with this one, so every later
// load (mailbox data, peer dt) is ordered after the observed flag.
__device__ inline unsigned long long p2p_acquire(const unsigned long long* f) {
  return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline double p2p_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_SYSTEM));
}
// (FP32 build: the halo values are floats; the dt words stay doubles)
__device__ inline float p2p_load(const float* p) {
  return __int_as_float((int)__hip_atomic_load((const unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// Multi-GPU exchange fused into the lean tile kernel (xGMI mailboxes, see
// hf2d_p2p_xchg for the layout and the parity argument).  Step s of a rank:
//   start  the dt slot already holds the global MIN (folded by the previous
//          kernel's last workgroup); tiles at the strip edges stage their
//          ghost column straight from the mailbox of parity s-1;
//   end    cells of the first / last owned column store their new lean
//          state into the neighbour's mailbox of parity s with
//          system-coherent stores and wait for their completion (vmcnt);
//          the last workgroup to finish (completion counter) sends this
//          rank's local dt MIN to every peer, publishes flag s, waits
//          (bounded) for the peers' flag s and folds their dt into the slot.
// One kernel per step and a single waiting workgroup, at the tail: no
// exchange kernel, no pack/unpack pass, no host involvement, and no
// system-scope fence (L2 writeback / invalidate) in the other workgroups.
// Ghost columns of the state arrays are only refreshed by
// hf2d_p2p_complete, which the host runs before any other consumer.
__device__ inline void p2p_store(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void p2p_store(float* p, float v) {
  __hip_atomic_store((unsigned*)p, (unsigned)__float_as_int(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// outstanding vector-memory operations of this wave (stores included on gfx9)
// have completed: the ordering point for the relaxed system-coherent stores
__device__ inline void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ inline unsigned long long rt_clock() { return __builtin_amdgcn_s_memrealtime(); }
constexpr int FX_DONE_STRIDE = 32;   // completion counters on lines of their own
// tail phase trace (HF2D_FX_SKIP bit 4, loopback timing runs only): after the
// counters, FX_TRACE_N records of FX_TRACE_W clocks, one per step (seq mod N)
constexpr int FX_TRACE_N = 64, FX_TRACE_W = 8;
constexpr unsigned FX_COUNT1_MAX = 512;
constexpr int FX_DONE_WORDS = (DT_SHARDS + 1) * FX_DONE_STRIDE + 2 * FX_TRACE_N * FX_TRACE_W;
struct FusedX {
  real* peer_recv_l;   // left neighbour's mailbox recv base (we are its right side)
  real* peer_recv_r;
  const real* my_recv;
  unsigned long long* const* peer_flags;
  double* const* peer_dtr;
  const unsigned long long* my_flags;
  const double* my_dtr;
  unsigned long long* seq;   // last published sequence number
  unsigned* done;            // workgroups finished in this step: per dt shard, then the shards (FX_DONE_STRIDE apart)
  long cap;
  int rank, nranks, sides, on;
  // lagged dt: the tail waits for the two neighbours' flags only and leaves
  // the dt MIN to the next step's first workgroup (lean_tile_body) or to
  // hf2d_p2p_complete
  int defer;
  // cost attribution of the fused exchange (HF2D_FX_SKIP, timing only, wrong
  // results): bit 0 no tail, bit 1 no edge pushes / mailbox stores, bit 2
  // ghosts staged from the state arrays instead of the mailbox (no ghost
  // prologue), bit 3 no loads of the push kernel
  int skip;
  int edge_first;   // inviscid fused tile kernel: edge tile columns dispatched first (HF2D_FX_EDGE_FIRST)
  // tail completion count: one per dt shard + one for the shards, or one
  // counter where the caller asks for it (fused lean N-S kernel, grids of <=
  // FX_COUNT1_MAX workgroups); HF2D_FX_COUNT1 = 1 / 2 forces one / two levels.
  // Loopback tail trace: the resonator's 4-rank strip (420 workgroups that
  // finish spread out) 0.96 -> 0.52 us of counting and 4.4 -> 3.4 us of
  // exchange with one counter; workgroups that finish together contend on it:
  // the headline's 8-rank strip (719 single-wave workgroups) 5.5 -> 11.7 us,
  // the scramjet's push kernel (135) 1.5 - 1.7 us of counting
  int count1;
};

// Peer waits and publications are spread over the lanes of one wavefront:
// lane q polls / publishes to peer q (q < nranks <= 64 per pass), so a step
// costs one round trip to the fine-grained mailbox per phase instead of one
// per peer (the single-thread loops cost ~12 us per step on an 8-rank strip,
// tools/exchange_loopback.py, profiles/exchange_loopback_r05.md).
__device__ inline double wave_min(double v) {
#pragma unroll
  for (int off = 1; off < WAVE; off <<= 1) v = fmin(v, __shfl_xor(v, off, WAVE));
  return v;
}
// Every lane of the calling wavefront: wait (bounded) for the flags of the
// peers q with need(q) to reach target (acquire), and return the MIN of
// their dt of parity par (fold) -- or 1.0 without fold.  False through *ok
// after a timeout (neg_T bit 2) or an earlier one.
template <class Need>
__device__ inline double p2p_wait_wave(const FusedX& x, unsigned long long target, DevScalars* sc, Need need,
                                       bool fold, int par, bool* ok) {
  const int lane = (int)(threadIdx.x & (WAVE - 1));
  bool good = !(__hip_atomic_load(&sc->neg_T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2);
  double d = 1.0;
  for (int q = lane; q < x.nranks && good; q += WAVE) {
    if (q == x.rank || !need(q)) continue;
    long spins = 0;
    while (__hip_atomic_load(&x.my_flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > P2P_SPIN_LIMIT) {
        atomicOr(&sc->neg_T, 2);
        good = false;
        break;
      }
    }
    // acquire the peer's publication: its dt and mailbox stores (released by
    // its vmcnt drain before the flag) are visible to every load ordered
    // after this one, here and in later kernels
    if (good) (void)p2p_acquire(&x.my_flags[q]);
    if (good && fold) d = fmin(d, p2p_load(x.my_dtr + par * x.nranks + q));
  }
  *ok = __ballot(!good) == 0;
  return wave_min(d);
}
__device__ inline bool p2p_wait_all(const FusedX& x, unsigned long long target, DevScalars* sc) {
  bool ok;
  (void)p2p_wait_wave(x, target, sc, [](int) { return true; }, false, 0, &ok);
  return ok;
}

// Tail of a step kernel with the exchange fused in (wavefront 0 of every
// workgroup, after the workgroup's mailbox stores and dt MIN): the last
// workgroup to finish publishes this rank's step (its dt to every peer, then
// flag seq_prev + 1), waits (bounded) for every peer's flag of the same step
// -- the two neighbours' only with X.defer -- and folds their dt into the
// slot the next step reads.
// Returns true (every lane) in the last workgroup, after the wait.
__device__ __forceinline__ bool fx_tail(const FusedX& X, DevScalars* sc, int slot_next,
                                        unsigned long long seq_prev, bool fold = true, bool one_level = false) {
  const int lane = (int)(threadIdx.x & (WAVE - 1));
  const bool trace = (X.skip & 16) != 0;
  unsigned long long c[FX_TRACE_W] = {};
  if (trace) c[0] = rt_clock();
  // the workgroup barrier drained every wave's mailbox stores; drain lane
  // 0's dt atomic before counting this workgroup as done
  vm_drain();
  if (trace) c[1] = rt_clock();
  // completion count in two levels (one counter per dt shard, then one for
  // the shards): a single counter serialises every workgroup's returning
  // atomic at the memory side
  int last = 0;
  if (lane == 0 && (X.count1 == 1 || (X.count1 == 0 && one_level))) {
    unsigned* ct = X.done + DT_SHARDS * FX_DONE_STRIDE;
    if (__hip_atomic_fetch_add(ct, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(ct, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = 1;
    }
  } else if (lane == 0) {
    const unsigned G = gridDim.x, sh = blockIdx.x % DT_SHARDS;
    const unsigned pop = (G - sh + DT_SHARDS - 1) / DT_SHARDS, nsh = G < DT_SHARDS ? G : DT_SHARDS;
    unsigned* cs = X.done + sh * FX_DONE_STRIDE;
    unsigned* ct = X.done + DT_SHARDS * FX_DONE_STRIDE;
    if (__hip_atomic_fetch_add(cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pop - 1) {
      __hip_atomic_store(cs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(ct, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1) {
        __hip_atomic_store(ct, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
  }
  if (!__shfl(last, 0, WAVE)) return false;
  if (trace) c[2] = rt_clock();
  // last workgroup: this rank's dt (word + shards, one per lane), published
  // to every peer (one peer per lane), then the flags, then the peers'
  const unsigned long long sn = seq_prev + 1;
  const int pn = (int)(sn & 1);
  unsigned long long b = ~0ull;
  if (lane < DT_SHARDS)
    b = __hip_atomic_load(&sc->dt_sh[slot_next][lane][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == DT_SHARDS) b = __hip_atomic_load(&sc->dt_bits[slot_next], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double d = wave_min(b == ~0ull ? 1.0 : bits_to_d(b));
  if (trace) c[3] = rt_clock();
  for (int q = lane; q < X.nranks; q += WAVE)
    if (q != X.rank) p2p_store(X.peer_dtr[q] + pn * X.nranks + X.rank, d);
  vm_drain();   // (the wavefront's stores: every lane's)
  if (trace) c[4] = rt_clock();
  for (int q = lane; q < X.nranks; q += WAVE)
    if (q != X.rank) __hip_atomic_store(&X.peer_flags[q][X.rank], sn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (trace) c[5] = rt_clock();
  const bool defer = X.defer != 0;
  const int r = X.rank;
  bool ok;
  const double peers = p2p_wait_wave(X, sn, sc, [=](int q) { return !defer || q == r - 1 || q == r + 1; },
                                     fold && !defer, pn, &ok);
  d = fmin(d, peers);
  if (trace) c[6] = rt_clock();
  if (lane == 0) {
    if (fold && !defer && ok)
      __hip_atomic_store(&sc->dt_bits[slot_next], d_to_bits(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *X.seq = sn;
    if (trace) {
      vm_drain();
      c[7] = rt_clock();
      unsigned long long* o = reinterpret_cast<unsigned long long*>(X.done + (DT_SHARDS + 1) * FX_DONE_STRIDE) +
                              (long)(sn % FX_TRACE_N) * FX_TRACE_W;
#pragma unroll
      for (int k = 0; k < FX_TRACE_W; k++) o[k] = c[k];
    }
  }
  return true;
}


// Single-GPU last step of a host call (StepParams::host_sc): the last
// workgroup to finish copies the slot's dt (word + shards) and the error flag
// into the pinned host mirror (workgroup 0's head wrote time_part / dt_lag
// there), so DeviceSolver::sync_scalars only waits for the stream: no
// hf2d_scalars_out launch and its completion round trip (13 us of an idle
// step(0) call, tools/call_overhead.py).  Completion count as fx_tail.
__device__ __forceinline__ void host_mirror_tail(const StepParams& P, DevScalars* sc, int slot_next) {
  const int lane = (int)(threadIdx.x & (WAVE - 1));
  vm_drain();   // lane 0's dt atomic
  int last = 0;
  if (lane == 0) {
    const unsigned G = gridDim.x, sh = blockIdx.x % DT_SHARDS;
    const unsigned pop = (G - sh + DT_SHARDS - 1) / DT_SHARDS, nsh = G < DT_SHARDS ? G : DT_SHARDS;
    unsigned* cs = P.host_done + sh * FX_DONE_STRIDE;
    unsigned* ct = P.host_done + DT_SHARDS * FX_DONE_STRIDE;
    if (__hip_atomic_fetch_add(cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pop - 1) {
      __hip_atomic_store(cs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(ct, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1) {
        __hip_atomic_store(ct, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
  }
  if (!__shfl(last, 0, WAVE)) return;
  unsigned long long b = ~0ull;
  if (lane < DT_SHARDS) b = __hip_atomic_load(&sc->dt_sh[slot_next][lane][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == DT_SHARDS) b = __hip_atomic_load(&sc->dt_bits[slot_next], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (P.dt_fold) {
    // the step's MIN into the slot's word: the next step reads one word
    // (StepParams::dt_read = 2) instead of the word and 16 shards
    unsigned long long m = b;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) m = dt_bits_min(m, (unsigned long long)__shfl_xor((long long)m, off, WAVE));
    m = (unsigned long long)__shfl((long long)m, 0, WAVE);
    if (lane == DT_SHARDS) {
      b = m;
      __hip_atomic_store(&sc->dt_bits[slot_next], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (!P.host_sc) return;
  DevScalars* h = static_cast<DevScalars*>(P.host_sc);
  if (lane <= DT_SHARDS) (lane < DT_SHARDS ? h->dt_sh[slot_next][lane][0] : h->dt_bits[slot_next]) = b;
  if (lane == DT_SHARDS + 1) h->neg_T = __hip_atomic_load(&sc->neg_T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (workgroup 0's head, thread 0, after its updates of the slot words)
__device__ __forceinline__ void host_mirror_head(const StepParams& P, const DevScalars* sc, int slot_next) {
  DevScalars* h = static_cast<DevScalars*>(P.host_sc);
  h->time_part = sc->time_part;
  h->dt_lag[slot_next] = sc->dt_lag[slot_next];
}

// LDS-tiled lean step (lean_euler.hpp: lean_tile_stage / TileIO).
// In-kernel phase trace (TR): thread 0 of every workgroup records the
// 100 MHz s_memrealtime clock at entry, after the LDS staging barrier, when
// its own wave finished computing, after the block dt reduction barrier and
// after the dt atomic, plus the HW_ID / XCC_ID registers (DeviceSolver::trace_tile).
constexpr int TILE_TRACE_WORDS = 8;
#ifndef HF2D_TILE_STAGGER
#define HF2D_TILE_STAGGER 1
#endif
constexpr int LDS_PER_CU = 160 * 1024;

// part: 0 every tile; 1 the tiles of the strip's first and last tile column
// (their results feed the halo exchange); 2 the other tiles.  The grid of a
// part launch has exactly that many workgroups (DeviceSolver comm overlap).
__device__ inline unsigned tile_of_part(unsigned bl, int part, const LeanTile& T) {
  if (part == 1) return bl < (unsigned)T.nbj ? bl : (unsigned)((T.nbi - T.ne) * T.nbj) + (bl - T.nbj);
  if (part == 2) return (unsigned)T.nbj + bl;
  return bl;
}

// all tiles, the strip's edge tile columns first (the first one, then the
// last T.ne), then the interior ones in order
__device__ inline unsigned tile_edge_first(unsigned bl, const LeanTile& T) {
  const unsigned nbj = (unsigned)T.nbj, ne = (unsigned)T.ne, nbi = (unsigned)T.nbi;
  if (nbi < 2 + ne || bl < nbj) return bl;
  if (bl < (1 + ne) * nbj) return (nbi - ne) * nbj + (bl - nbj);
  return nbj + (bl - (1 + ne) * nbj);
}

// NT: threads per workgroup (BLOCK, or 128 / 64 for the small strips of a
// multi-GPU run: at 250 x 200 cells per GPU a 256-thread tiling leaves ~50 of
// the 256 CUs without a workgroup, and the step is one workgroup's
// load -> compute -> reduce chain)
template <bool RES, bool OUT, bool SG, int CPT, bool FX = false, bool TR = false, int NT = BLOCK>
__device__ __forceinline__ void lean_tile_body(StepParams& P, const LeanSoA& L, const LeanTile& T, DevScalars* sc,
                                               int slot, int slot_next, int serial, ResidualPack* partials,
                                               const FusedX& X = FusedX{}, unsigned long long* trace = nullptr,
                                               int part = 0) {
  extern __shared__ real lds[];
  unsigned long long tr[5];
  if (TR) tr[0] = rt_clock();
  // (compiled into the single-gas two-cell kernel only: the mere presence of
  // this block made the multi-gas one-cell kernel 3x slower on the triple
  // point, 340 -> 1030 us, even with stagger 0)
  if (HF2D_TILE_STAGGER && SG && CPT == 2 && !FX && NT == BLOCK && P.stagger != 0) {
    // staggered start: every workgroup of a step is resident at once, so
    // without it they all stage together (HBM saturated, VALUs idle) and
    // then all compute (HBM idle); later dispatch rounds start loading while
    // the earlier ones compute
    // (rounds beyond the 4th are dispatched as earlier workgroups retire:
    // no wait for them)
    // (stagger > 0: whole rounds of stagger_wgs workgroups; < 0: a linear
    // ramp of the same slope over the first four rounds)
    const unsigned r = blockIdx.x / (unsigned)P.stagger_wgs;
    if (r < 4 && (P.stagger < 0 || r > 0)) {
      const unsigned long long d = P.stagger > 0 ? (unsigned long long)r * (unsigned)P.stagger
                                                 : (unsigned long long)blockIdx.x * (unsigned)(-P.stagger) /
                                                       (unsigned)P.stagger_wgs;
      const unsigned long long t0 = rt_clock();
      while (rt_clock() - t0 < d) __builtin_amdgcn_s_sleep(2);
    }
  }
  // (fused exchange: the strip's edge tile columns first -- they push the
  // halo and stage the ghost columns from the mailbox)
  const unsigned b = (FX && X.edge_first) ? tile_edge_first(xcd_remap(blockIdx.x, gridDim.x), T)
                                          : tile_of_part(xcd_remap(blockIdx.x, gridDim.x), part, T);
  unsigned long long seq_prev = 0;
  if (FX) seq_prev = *X.seq;
  apply_dt(P, sc, slot, true);
  if (b == 0 && threadIdx.x < WAVE) {
    // lagged dt with the fold deferred (X.defer): the previous step's tail
    // waited for the two neighbours only; the other ranks' dt of that step
    // is folded here, one step later, by this wavefront (one peer per lane)
    double fold = 1.0;
    if (FX && X.defer && P.lag_dt && seq_prev > 0) {
      bool ok;
      fold = p2p_wait_wave(X, seq_prev, sc, [](int) { return true; }, true, (int)(seq_prev & 1), &ok);
    }
    if (threadIdx.x == 0) {
      dt_reset(sc, slot_reset(slot));
      lag_head(P, sc, slot, slot_next, fold);
      sc->dt_bits[slot] = d_to_bits(P.dt);   // folded (later kernels of the step read the word)
      sc->time_part += P.dt;
      scenario_next(P, sc, slot, slot_next);
      if (OUT && !RES && !FX && P.host_sc) host_mirror_head(P, sc, slot_next);
    }
  }
  int i[CPT], j[CPT], c[CPT], i0, j0;
  bool mine[CPT];
  // own-cell global inputs first, so they are in flight during the staging
  LeanOwn own[CPT];
#pragma unroll
  for (int q = 0; q < CPT; q++) {
    mine[q] = lean_tile_cell(P, T, (int)b, (int)threadIdx.x, &i[q], &j[q], &c[q], &i0, &j0, q);
    if (mine[q]) lean_load_own<TileIO<SG>::NE>(L, (long)i[q] * P.ny + j[q], own[q]);
  }
  if (!FX || seq_prev == 0 || (X.skip & 4) || (i0 - 1 > P.i0 - 1 && i0 + T.TI < P.i1)) {
    lean_tile_stage<SG>(P, L, T, i0, j0, lds, threadIdx.x, NT);
  } else {
    // edge tile: the ghost column comes from the mailbox of parity seq_prev
    constexpr int NF = SG ? LEAN_TILE_FIELDS_SG : LEAN_TILE_FIELDS;
    const int pp = (int)(seq_prev & 1);
    const real* mbL = X.my_recv + ((long)pp * 2) * X.cap;
    const real* mbR = X.my_recv + ((long)pp * 2 + 1) * X.cap;
    const long N = L.N;
    constexpr int NS = SG ? 4 : 4 + NCOMP;
    constexpr int FU = SG ? 4 : 10;
    for (int c = threadIdx.x; c < T.NC; c += NT) {
      const int ii = c / T.W - 1, jj = c - (ii + 1) * T.W - 1;
      const bool xh = ii < 0 || ii >= T.TI, yh = jj < 0 || jj >= T.TJ;
      const int gi = i0 + ii, gj = j0 + jj;
      if ((xh && yh) || gi < 0 || gi >= P.nx || gj < 0 || gj >= P.ny) continue;
      const bool gl = (X.sides & 1) && gi == P.i0 - 1, gr = (X.sides & 2) && gi == P.i1;
      if (gl || gr) {
        const real* mb = gl ? mbL : mbR;
#pragma unroll
        for (int f = 0; f < NF; f++) lds[f * T.NC + c] = p2p_load(mb + (long)f * P.ny + gj);
        continue;
      }
      const long g = (long)gi * P.ny + gj;
#pragma unroll
      for (int f = 0; f < NS; f++) lds[f * T.NC + c] = L.Sin[f * N + g];
      if (!SG)
#pragma unroll
        for (int f = 0; f < NCOMP; f++) lds[(4 + NCOMP + f) * T.NC + c] = L.Pin_s[f * N + g];
      lds[FU * T.NC + c] = L.Uin[g];
      lds[(FU + 1) * T.NC + c] = L.Vin[g];
      lds[(FU + 2) * T.NC + c] = L.Pin[g];
    }
  }
  __syncthreads();
  // (raising the wave priority here for the compute phase, s_setprio 2,
  // measured no change: headline 26.9 - 27.2 us either way, triple point
  // 350 - 353 us)
  if (TR) tr[1] = rt_clock();
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  double dtl = 1.0;
  int neg = 0;
#pragma unroll
  for (int q = 0; q < CPT; q++) {
    if (mine[q]) {
      TileIO<SG> io(L, (long)i[q] * P.ny + j[q], lds, T.NC, T.W, c[q]);
      dtl = fmin(dtl, lean_cell<RES, OUT>(P, L, io, own[q], i[q], j[q], r, &neg));
      if (FX) {
        const bool pl = (X.sides & 1) && i[q] == P.i0, pr = (X.sides & 2) && i[q] == P.i1 - 1;
        if ((pl || pr) && !(X.skip & 2)) {   // new lean state of an edge cell -> the neighbour's mailbox of parity seq_prev + 1
          constexpr int NF = SG ? LEAN_TILE_FIELDS_SG : LEAN_TILE_FIELDS;
          constexpr int NS = SG ? 4 : 4 + NCOMP;
          const int pn = (int)((seq_prev + 1) & 1);
          real* mb = pl ? X.peer_recv_l + ((long)pn * 2 + 1) * X.cap : X.peer_recv_r + ((long)pn * 2) * X.cap;
          const long N = L.N, g = (long)i[q] * P.ny + j[q];
          real v[NF];
#pragma unroll
          for (int f = 0; f < NS; f++) v[f] = L.Sout[f * N + g];
          if (!SG)
#pragma unroll
            for (int f = 0; f < NCOMP; f++) v[4 + NCOMP + f] = L.Pout_s[f * N + g];
          v[NF - 3] = L.Uout[g];
          v[NF - 2] = L.Vout[g];
          v[NF - 1] = L.Pout[g];
#pragma unroll
          for (int f = 0; f < NF; f++) p2p_store(mb + (long)f * P.ny + j[q], v[f]);
          vm_drain();
        }
      }
    }
  }
  if (TR) tr[2] = rt_clock();
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)b * (NT / WAVE) + threadIdx.x / WAVE] = r;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[NT / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) {
    atomicOr(&sc->neg_T, 1);
    if (OUT && !RES && !FX && P.host_sc) vm_drain();   // (done before host_mirror_tail's count)
  }
  __syncthreads();
  if (TR) tr[3] = rt_clock();
  if (threadIdx.x == 0) {
    double m = sdt[0];
    for (int q = 1; q < NT / WAVE; q++) m = fmin(m, sdt[q]);
    if (serial) m = fmin(m, P.dt);
    dt_min(sc, slot_next, m);
    if (TR) {
      vm_drain();
      tr[4] = rt_clock();
      unsigned long long* o = trace + (long)b * TILE_TRACE_WORDS;
#pragma unroll
      for (int q = 0; q < 5; q++) o[q] = tr[q];
      o[5] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave/SIMD/CU/SE
      o[6] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
      o[7] = blockIdx.x;
    }
  }
  if (FX && threadIdx.x < WAVE && !(X.skip & 1)) fx_tail(X, sc, slot_next, seq_prev);
  if (!FX && !TR && (P.dt_fold || (OUT && !RES && P.host_sc)) && threadIdx.x < WAVE)
    host_mirror_tail(P, sc, slot_next);
}

// No occupancy attribute on the default kernel: the backend's own register
// budget (94 VGPRs here) beat every explicit amdgpu_waves_per_eu we tried.
template <bool RES, bool OUT, bool SG, int OCC = 0, int CPT = 1>
__global__ __launch_bounds__(BLOCK) void hf2d_lean_tile(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                         int slot, int slot_next, int serial,
                                                         ResidualPack* partials, int part = 0) {
  lean_tile_body<RES, OUT, SG, CPT>(P, L, T, sc, slot, slot_next, serial, partials, FusedX{}, nullptr, part);
}

// Phase-traced plain step (profiling only, DeviceSolver::trace_tile).
template <bool SG, int CPT>
__global__ __launch_bounds__(BLOCK) void hf2d_lean_tile_tr(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                            int slot, int slot_next, int serial,
                                                            ResidualPack* partials, unsigned long long* trace) {
  lean_tile_body<false, false, SG, CPT, false, true>(P, L, T, sc, slot, slot_next, serial, partials, FusedX{}, trace);
}

// Same step with the multi-GPU exchange fused in (FusedX).
template <bool RES, bool OUT, bool SG, int CPT>
// (the exchange arguments by pointer, read where they are used: by value
// they took ~26 SGPRs of the kernel arguments, and the 64-thread fused
// kernel spilled 96 SGPRs to VGPR lanes against 28 for the plain one)
__global__ __launch_bounds__(BLOCK) void hf2d_lean_tile_fx(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                            int slot, int slot_next, int serial,
                                                            ResidualPack* partials, const FusedX* __restrict__ X) {
  lean_tile_body<RES, OUT, SG, CPT, true>(P, L, T, sc, slot, slot_next, serial, partials, *X);
}

// Small-strip geometries (single gas): NT = 128 / 64 threads per workgroup
// (picked by the ThreadBlockSize = 0 autotune per strip)
template <bool RES, bool OUT, int NT, int CPT>
__global__ __launch_bounds__(NT) void hf2d_lean_tile_nt(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                       int slot, int slot_next, int serial, ResidualPack* partials,
                                                       int part = 0) {
  lean_tile_body<RES, OUT, true, CPT, false, false, NT>(P, L, T, sc, slot, slot_next, serial, partials, FusedX{},
                                                        nullptr, part);
}
template <bool RES, bool OUT, int NT, int CPT>
__global__ __launch_bounds__(NT) void hf2d_lean_tile_fx_nt(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                          int slot, int slot_next, int serial,
                                                          ResidualPack* partials, const FusedX* __restrict__ X) {
  lean_tile_body<RES, OUT, true, CPT, true, false, NT>(P, L, T, sc, slot, slot_next, serial, partials, *X);
}
template <int NT, int CPT>
__global__ __launch_bounds__(NT) void hf2d_lean_tile_tr_nt(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc,
                                                          int slot, int slot_next, int serial,
                                                          ResidualPack* partials, unsigned long long* trace) {
  lean_tile_body<false, false, true, CPT, false, true, NT>(P, L, T, sc, slot, slot_next, serial, partials, FusedX{},
                                                           trace);
}

// Ghost columns + global dt after fused steps, for any other consumer: wait
// for the peers' last publication, copy the mailbox of that parity into the
// ghost columns of the current state, fold the dt MIN into the slot.
__global__ __launch_bounds__(P2P_THREADS) void hf2d_p2p_complete(ColList Lc, int ghostL, int ghostR, int ny, int cnt,
                                                                 FusedX X, DevScalars* sc, int dslot) {
  const unsigned long long sq = *X.seq;
  if (sq == 0) return;
  __shared__ int ok;
  if (threadIdx.x < WAVE) {
    const bool w = p2p_wait_all(X, sq, sc);
    if (threadIdx.x == 0) ok = w ? 1 : 0;
  }
  __syncthreads();
  if (!ok) return;
  const int pp = (int)(sq & 1);
  if (X.sides & 1) {
    const real* src = X.my_recv + ((long)pp * 2) * X.cap;
    for (int t = threadIdx.x; t < cnt; t += P2P_THREADS) {
      const int f = t / ny, j = t - f * ny;
      Lc.f[f][(long)ghostL * ny + j] = p2p_load(src + t);
    }
  }
  if (X.sides & 2) {
    const real* src = X.my_recv + ((long)pp * 2 + 1) * X.cap;
    for (int t = threadIdx.x; t < cnt; t += P2P_THREADS) {
      const int f = t / ny, j = t - f * ny;
      Lc.f[f][(long)ghostR * ny + j] = p2p_load(src + t);
    }
  }
  if (threadIdx.x == 0) {
    double m = dt_get(sc, dslot);
    for (int q = 0; q < X.nranks; q++)
      if (q != X.rank) m = fmin(m, p2p_load(X.my_dtr + pp * X.nranks + q));
    sc->dt_bits[dslot] = d_to_bits(m);
  }
}

template <bool RES, bool OUT, bool SG, int OCC, int CPT = 1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(OCC)))
void hf2d_lean_tile_occ(StepParams P, LeanSoA L, LeanTile T, DevScalars* sc, int slot, int slot_next, int serial,
                        ResidualPack* partials) {
  lean_tile_body<RES, OUT, SG, CPT>(P, L, T, sc, slot, slot_next, serial, partials);
}

// K8 monitors: p and Tg of the probe cells this rank owns (idx < 0: not
// owned) gathered on the device, so an output step moves 16 bytes per probe
// instead of the whole state.
__global__ void hf2d_probe_gather(const long* idx, int n, const real* p, const real* T, real* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const long c = idx[t];
  out[2 * t] = c >= 0 ? p[c] : 0.0;
  out[2 * t + 1] = c >= 0 ? T[c] : 0.0;
}

__global__ __launch_bounds__(BLOCK) void hf2d_lean_materialize(StepParams P, LeanSoA L, SoA g, long c0, long c1) {
  const long c = c0 + (long)blockIdx.x * BLOCK + threadIdx.x;
  if (c >= c1) return;
  const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
  lean_materialize_cell(P, L, g, i, j);
}

// ---------------------------------------------------------------------------
// Lean single-gas N-S step (lean_ns.hpp): F_m of the tile + ring into LDS,
// predict_m from LDS, own-cell part of F_{m+1} for dt_{m+1}.  One workgroup
// per TI x TJ tile (lean_tile_geom, one cell per thread).
// ---------------------------------------------------------------------------
constexpr int LNS_SKIP_ERR = 8;   // neg_T bit: fill_node() skipped a node (rho == 0 or k < 1)

// Ghost prologue of a fused lean N-S / mechanism step (replaces the separate
// hf2d_p2p_unpack launch after the previous fused step): a tile whose fills
// read a ghost column copies the rows it reads, [j0 - 1, j0 + TJ], of every
// HALO_LNS entry of the previous step's list Lg from this rank's mailbox of
// parity seq_prev (the previous kernel's tail acquired the peers' flags) into
// the ghost columns; the workgroup barrier makes them visible to its own
// loads.  Vertically adjacent edge tiles write the rows they share with the
// same values, and every ghost value a tile reads it wrote itself: a
// workgroup reads its own stores through its CU's L1 (workgroup-scope
// coherence needs no cache maintenance outside thread-group-split mode; an
// agent-scope acquire here invalidates the XCD's L2 lines and measured
// 14.8 -> 23.3 us of exchange cost on the 4-rank Step strip).
__device__ inline void fx_ghost_prologue(const StepParams& P, const FusedX& X, const ColList* Lg, int i0, int j0,
                                         int TI, int TJ, unsigned long long seq_prev) {
  const bool gl = (X.sides & 1) && i0 <= P.i0 + 1;
  const bool gr = (X.sides & 2) && i0 + TI + 1 >= P.i1;
  if (!gl && !gr) return;
  const int par = (int)(seq_prev & 1), nf = Lg->nf;
  const int jlo = j0 > 0 ? j0 - 1 : 0, jhi = j0 + TJ + 1 < P.ny ? j0 + TJ + 1 : P.ny;
  const int rows = jhi - jlo, per_side = nf * rows;
  for (int t = (int)threadIdx.x; t < 2 * per_side; t += (int)blockDim.x) {
    const int side = t < per_side ? 0 : 1;
    if (side == 0 ? !gl : !gr) continue;
    const int tt = t - side * per_side, f = tt / rows, j = jlo + (tt - f * rows);
    const real v = p2p_load(X.my_recv + ((long)par * 2 + side) * X.cap + (long)f * P.ny + j);
    Lg->f[f][(long)(side == 0 ? P.i0 - 1 - Lg->o[f] : P.i1 + Lg->o[f]) * P.ny + j] = v;
  }
  __syncthreads();
}

// Edge push of a fused lean N-S step, by every thread of an edge tile after
// the tile's barrier: the HALO_LNS values of the tile's cells in the strip's
// first / last two columns (entry f of Lc at column P.i0 + o[f] / P.i1 - 1 -
// o[f], stored by their owner threads before the barrier) -> the neighbour's
// mailbox of parity seq_prev + 1, K independent loads then K stores per
// thread; drained, then a barrier, so the tail counts a workgroup whose
// mailbox stores have completed.  (The owner threads pushing their own
// cells -- one column of 20 threads per offset, ~20 fields each -- kept the
// edge tiles, the last to finish in a one-round grid, ~4.6 us longer on the
// resonator's 4-rank strip, tools/exchange_loopback.py.)
__device__ inline void fx_edge_push(const StepParams& P, const FusedX& X, const ColList* Lc, const LeanTile& T, int i0,
                                    int j0, unsigned long long seq_prev) {
  const bool el = (X.sides & 1) && i0 <= P.i0 + 1;
  const bool er = (X.sides & 2) && i0 + T.TI >= P.i1 - 1;
  if (!el && !er) return;   // (uniform over the workgroup)
  const int pn = (int)((seq_prev + 1) & 1);
  const int jhi = j0 + T.TJ < P.ny ? j0 + T.TJ : P.ny, rows = jhi - j0, nf = Lc->nf;
  const int per = nf * rows, total = (el && er ? 2 : 1) * per;
  constexpr int K = 4;
  for (int base = (int)threadIdx.x; base < total; base += K * BLOCK) {
    real v[K];
    real* dst[K];
#pragma unroll
    for (int u = 0; u < K; u++) {
      const int t = base + u * BLOCK;
      dst[u] = nullptr;
      v[u] = 0.0;
      if (t < total) {
        const int side = (el && er) ? t / per : (el ? 0 : 1);
        const int tt = (el && er) ? t - side * per : t, f = tt / rows, j = j0 + (tt - f * rows), o = Lc->o[f];
        const int col = side == 0 ? P.i0 + o : P.i1 - 1 - o;
        if (col >= i0 && col < i0 + T.TI && col >= P.i0 && col < P.i1) {
          dst[u] = (side == 0 ? X.peer_recv_l + ((long)pn * 2 + 1) * X.cap : X.peer_recv_r + ((long)pn * 2) * X.cap) +
                   (long)f * P.ny + j;
          v[u] = Lc->f[f][(long)col * P.ny + j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < K; u++)
      if (dst[u]) p2p_store(dst[u], v[u]);
  }
  vm_drain();
  __syncthreads();
}

// FX: the multi-GPU exchange fused in (xGMI mailboxes): the cells of the
// strip's first / last two columns store this step's HALO_LNS values (Lc:
// the post-step pointers, DeviceSolver::halo_list) into the neighbour's
// mailbox, the last workgroup publishes the step and folds the peers' dt
// (fx_tail); hf2d_p2p_unpack then fills the ghost columns.
template <bool RES, int MODE, int TURB, bool FX = false>
__device__ __forceinline__ void lns_step_body(StepParams& P, const LnsArrays& a, const LeanTile& T, DevScalars* sc,
                                              int slot, int slot_next, int serial, ResidualPack* partials,
                                              int part, const FusedX& X = FusedX{}, const ColList* Lc = nullptr,
                                              const ColList* Lg = nullptr) {
  extern __shared__ real lds[];
  constexpr int NL = Lns<MODE>::NL;
  unsigned long long seq_prev = 0;
  if (FX) seq_prev = *X.seq;
  // part: 0 every tile, 1 / 2 the edge / interior tiles (comm overlap)
  // (a ghost prologue delays the strip's edge tiles: they go first, so they
  // do not finish the kernel late)
  const unsigned b = (FX && Lg != nullptr) ? tile_edge_first(xcd_remap(blockIdx.x, gridDim.x), T)
                                           : tile_of_part(xcd_remap(blockIdx.x, gridDim.x), part, T);
  apply_dt(P, sc, slot);
  if (b == 0 && threadIdx.x == 0) {
    dt_reset(sc, slot_reset(slot));
    lag_head(P, sc, slot, slot_next);
    sc->dt_bits[slot] = d_to_bits(P.dt);   // folded (later kernels of the step read the word)
    sc->time_part += P.dt;
    sc->dt_val[slot] = P.dt;
    scenario_next(P, sc, slot, slot_next);
  }
  // F_m runs with the dt of the step the split fill F_m belongs to (SST's
  // point-implicit destruction reads it); the predictor with this step's
  // (both read here: a second read of the device scalars after the fills
  // made the whole kernel 2x slower)
  const real dt_now = P.dt;
  if (MODE == SK_SGT && TURB == 3) P.dt = sc->dt_val[slot_reset(slot)];
  const int NC = T.NC;
  int i, j, c, i0, j0;
  const bool mine = lean_tile_cell(P, T, (int)b, (int)threadIdx.x, &i, &j, &c, &i0, &j0);
  int dummy = 0, skip = 0;
  // 0. the previous fused step's halo from the mailbox into the ghost columns
  if (FX && Lg != nullptr && seq_prev > 0 && !(X.skip & 4)) fx_ghost_prologue(P, X, Lg, i0, j0, T.TI, T.TJ, seq_prev);
  // 1a. ring cells first (only their S, A, B are kept)
  const int nring = 2 * (T.TI + T.TJ);
  // 1a'. a strip's first ghost column inside a partial last tile: its fill
  // is a neighbour's (the ring covers it when the tile is full).  One call
  // site for both (an inlined second copy of the fill costs registers).
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    int gi = -1, gj = 0, cc = 0;
    if (pass == 0) {
      if ((int)threadIdx.x < nring) {
        int ii, jj;
        lns_ring_cell(T, (int)threadIdx.x, &ii, &jj);
        gi = i0 + ii;
        gj = j0 + jj;
        cc = (ii + 1) * T.W + jj + 1;
      }
    } else if (!mine && (int)threadIdx.x < T.TIh * T.TJ && i == P.i1 && i < P.nx && j < P.ny) {
      gi = i;
      gj = j;
      cc = c;
    }
    if (gi >= 0 && gi < P.nx && gj >= 0 && gj < P.ny) {
      CellLocal rc;
      bool early, filled;
      lns_fill_to_lds<MODE, TURB>(P, a, gi, gj, lds, NC, cc, rc, &early, &filled, &dummy);
    }
  }
  // 1b. own cell: F_m, its level-m outputs, kept values for 2./3.
  LnsLevel<MODE> lv;
  u64 CT = 0, TT = 0;
  uint8_t gf = 0, nbm = 0;
  bool early = true, filled = false;
  const long N = a.N;
  const long idx = (long)i * P.ny + j;
  real bpre[NL];
  if (mine) {
#pragma unroll
    for (int q = 0; q < NL; q++) bpre[q] = a.beta[Lns<MODE>::eqk(q) * N + idx];
    CellLocal oc;
    lns_fill_to_lds<MODE, TURB>(P, a, i, j, lds, NC, c, oc, &early, &filled, &dummy);
    CT = oc.CT;
    gf = a.gf[idx];
    nbm = a.nb[idx];
    TT = a.TT[idx];
    if (!early) {
      if (!filled) skip = 1;
      a.Uo[idx] = oc.U;
      a.Vo[idx] = oc.V;
      a.To[idx] = oc.Tg;
      a.kko[idx] = oc.k;
      a.CPo[idx] = oc.CP;
      a.lamo[idx] = oc.lam;
      a.muo[idx] = oc.mu;
      if (MODE == SK_SGT) {
        a.mu_to[idx] = oc.mu_t;
        a.Src[(long)I_K * N + idx] = oc.Src[I_K];
        a.Src[(long)I_EPS * N + idx] = oc.Src[I_EPS];
      }
      if (gf & GF_SRCADD)
#pragma unroll
        for (int q = 0; q < NL; q++) {
          const int k = Lns<MODE>::eqk(q);
          a.SrcAdd[k * N + idx] = oc.SrcAdd[k];
        }
      lv.U = oc.U;
      lv.V = oc.V;
      lv.Tg = oc.Tg;
      lv.p = oc.p;
      lv.k = oc.k;
      lv.R = oc.R;
      lv.CP = oc.CP;
      lv.lam = oc.lam;
      lv.mu = oc.mu;
      lv.mu_t = oc.mu_t;
      lv.l_min = oc.l_min;
      lv.y_plus = oc.y_plus;
      lv.BGX = oc.BGX;
      lv.BGY = oc.BGY;
#pragma unroll
      for (int q = 0; q < NL; q++) {
        const int k = Lns<MODE>::eqk(q);
        lv.SrcAdd[q] = oc.SrcAdd[k];
        lv.F[q] = oc.F[k];
        lv.Src[q] = oc.Src[k];
      }
    }
  }
  P.dt = dt_now;   // this step's dt for the predictor
  __syncthreads();
  // 2. predict_m
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  double dtl = 1.0;
  int neg = 0;
  if (mine) {
    LnsPredictIO<MODE> io{a, lds, lv, bpre, N, idx, idx, idx, idx, idx, NC, c, c, c, c, c, gf, {}};
    if (!is_active(CT)) {
#pragma unroll
      for (int q = 0; q < NL; q++) {
        const int k = Lns<MODE>::eqk(q);
        io.sn[k] = io.S(k);
        io.keep_dS(k);
      }
    } else {
      const int n1 = (nbm & NB_XL) ? 1 : 0, n2 = (nbm & NB_XR) ? 1 : 0;
      const int n3 = (nbm & NB_YU) ? 1 : 0, n4 = (nbm & NB_YD) ? 1 : 0;
      io.iL = (long)(i - n1) * P.ny + j;
      io.iR = (long)(i + n2) * P.ny + j;
      io.iU = idx + n3;
      io.iD = idx - n4;
      io.cL = c - n1 * T.W;
      io.cR = c + n2 * T.W;
      io.cU = c + n3;
      io.cD = c - n4;
      predict_core<RES>(P, io, CT, TT, n1, n2, n3, n4, P.gx0 + i, j, r);
    }
#pragma unroll
    for (int q = 0; q < NL; q++) {
      const int k = Lns<MODE>::eqk(q);
      a.Sp_out[k * N + idx] = io.sn[k];
    }
    // 3. own-cell part of F_{m+1}: dt_{m+1}
    if (!early) {
      LnsOwnIO<MODE> oio(io.sn, lv, CT, TT, gf, nbm);
      CellLocal nc;
      real mY[1], mgx[1], mgy[1];
      bool e2, f2;
      dtl = fill_compute<MODE, 1, LnsOwnIO<MODE>, true>(P, oio, nc, mY, mgx, mgy, nullptr, 0, i, j, true, &neg, &e2,
                                                         &f2);
    }
  }
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)b * (BLOCK / WAVE) + threadIdx.x / WAVE] = r;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  if (skip) atomicOr(&sc->neg_T, LNS_SKIP_ERR);
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) m = fmin(m, sdt[q]);
    if (serial) m = fmin(m, P.dt);
    dt_min(sc, slot_next, m);
  }
  if (FX && !(X.skip & 2)) fx_edge_push(P, X, Lc, T, i0, j0, seq_prev);
  // (unpacking the peers' halo in this last workgroup instead of a separate
  // hf2d_p2p_unpack launch measured 2x the exchange cost: one workgroup's
  // serial rounds of uncached mailbox loads, profiles/exchange_loopback_r05.md)
  if (FX && threadIdx.x < WAVE && !(X.skip & 1)) fx_tail(X, sc, slot_next, seq_prev, true, gridDim.x <= FX_COUNT1_MAX);
}

// (LnsArrays by value: passed by device pointer instead, the k-eps
// kernel spilled 215 instead of 254 SGPRs but the resonator ran 2.5 % and
// Step 3.8 % slower: the fields were re-loaded inside the fills)
template <bool RES, int MODE, int TURB = 2>
__global__ __launch_bounds__(BLOCK) void hf2d_lns_step(StepParams P, LnsArrays a, LeanTile T, DevScalars* sc,
                                                        int slot, int slot_next, int serial, ResidualPack* partials,
                                                        int part) {
  lns_step_body<RES, MODE, TURB>(P, a, T, sc, slot, slot_next, serial, partials, part);
}
// the same step with the xGMI mailbox exchange fused in (the register
// budgets of the default kernels: laminar unbounded, k-eps / SST / SA 3
// waves per SIMD)
// (FusedX and the halo column list by device pointer, as the fused tile
// kernels: SGPR spills 170 -> 252 and the resonator's 4-rank loopback
// exchange 15.8 -> 16.5 us; kept by value)
template <bool RES, int MODE, int TURB>
__global__ __launch_bounds__(BLOCK) void hf2d_lns_step_fx(StepParams P, LnsArrays a, LeanTile T, DevScalars* sc,
                                                           int slot, int slot_next, int serial,
                                                           ResidualPack* partials, FusedX X, ColList Lc,
                                                           const ColList* Lg) {
  lns_step_body<RES, MODE, TURB, true>(P, a, T, sc, slot, slot_next, serial, partials, 0, X, &Lc, Lg);
}
template <bool RES, int MODE, int TURB>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(3))) void hf2d_lns_step_fx3(
    StepParams P, LnsArrays a, LeanTile T, DevScalars* sc, int slot, int slot_next, int serial,
    ResidualPack* partials, FusedX X, ColList Lc, const ColList* Lg) {
  lns_step_body<RES, MODE, TURB, true>(P, a, T, sc, slot, slot_next, serial, partials, 0, X, &Lc, Lg);
}

// Multi-workgroup mailbox exchange, push half (the mechanism step and every
// other p2p exchange with p2p_fuse): each thread loads up to PER boundary
// values of the fields in Lc (column first + o / last - o) and stores them
// into the neighbours' mailboxes; the last workgroup publishes and, fold,
// folds the peers' dt into dslot (fx_tail); hf2d_p2p_unpack follows.
// publish = 0: the pushes only (drained); a later hf2d_p2p_finish publishes
// the step -- the mechanism step pushes its edge tiles' halo before its
// interior tiles run.
template <int PER>
__global__ __launch_bounds__(BLOCK) void hf2d_p2p_push(ColList Lc, int first, int last, int ny, int cnt, FusedX X,
                                                      DevScalars* sc, int dslot, int fold, int publish) {
  const unsigned long long seq_prev = *X.seq;
  const int pn = (int)((seq_prev + 1) & 1);
  // value u of a thread: base + u * BLOCK (consecutive lanes, consecutive
  // addresses: with PER consecutive values per thread every load and mailbox
  // store instruction touched 64 different lines)
  const long base = (long)blockIdx.x * BLOCK * PER + threadIdx.x;
  real v[PER];
#pragma unroll
  for (int u = 0; u < PER; u++) {
    const long t = base + (long)u * BLOCK;
    if (t < 2L * cnt) {
      const int side = t < cnt ? 0 : 1;
      const int tt = (int)(t - (long)side * cnt), f = tt / ny, j = tt - f * ny;
      if ((X.sides & (1 << side)) && !(X.skip & 8))
        v[u] = Lc.f[f][(long)(side == 0 ? first + Lc.o[f] : last - Lc.o[f]) * ny + j];
    }
  }
#pragma unroll
  for (int u = 0; u < PER; u++) {
    const long t = base + (long)u * BLOCK;
    if (t < 2L * cnt) {
      const int side = t < cnt ? 0 : 1;
      const int tt = (int)(t - (long)side * cnt);
      // the left neighbour receives "from right", the right one "from left"
      if ((X.sides & (1 << side)) && !(X.skip & 2))
        p2p_store((side == 0 ? X.peer_recv_l + ((long)pn * 2 + 1) * X.cap : X.peer_recv_r + ((long)pn * 2) * X.cap) +
                      tt,
                  v[u]);
    }
  }
  vm_drain();
  if (!publish) return;
  __syncthreads();
  if (threadIdx.x < WAVE && !(X.skip & 1)) fx_tail(X, sc, dslot, seq_prev, fold != 0);
}

using PushK = void (*)(ColList, int, int, int, int, FusedX, DevScalars*, int, int, int);
// values per thread of the push kernel (HF2D_PUSH_PER: 1, 4 or 16) and its
// grid: one value per thread (135 workgroups on the scramjet's 8-rank strip)
// pushed the 43-field mechanism halo in 7.0 us against 15.4 us with 16 values
// per thread on 9 workgroups (rocprofv3 kernel trace of tools/exchange_loopback.py;
// loopback exchange 18.7 -> 8.2 us)
inline PushK push_kernel(int per) {
  return per == 16 ? hf2d_p2p_push<16> : per == 4 ? hf2d_p2p_push<4> : hf2d_p2p_push<1>;
}
inline unsigned push_grid(int per, int cnt) {
  const int p = per == 16 || per == 4 ? per : 1;
  return (unsigned)std::max(1, (2 * cnt + BLOCK * p - 1) / (BLOCK * p));
}

// One workgroup: publish the step whose halo an earlier hf2d_p2p_push
// (publish = 0) stored, wait for the peers' publication, fold their dt.
__global__ void hf2d_p2p_finish(FusedX X, DevScalars* sc, int dslot) {
  fx_tail(X, sc, dslot, *X.seq, true);   // (one wavefront)
}

// The scalars the host reads (the words before the dt shards, and the shards
// of the dt slot it reads) into pinned host memory with plain vector stores,
// queued behind the step's kernels: the host then waits for the stream only,
// instead of for the stream and a device-to-host copy of the whole block behind
// it (one copy-engine round trip per sync_scalars, i.e. per run_steps call).
__global__ __launch_bounds__(WAVE) void hf2d_scalars_out(const DevScalars* sc, DevScalars* host, int slot) {
  constexpr int NH = (int)(offsetof(DevScalars, dt_sh) / 8);
  static_assert(offsetof(DevScalars, dt_sh) % 8 == 0 && NH <= WAVE, "DevScalars header is copied in 8-byte words");
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(sc);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(host);
  const int t = threadIdx.x;
  if (t < NH) dst[t] = src[t];
  if (t < DT_SHARDS) host->dt_sh[slot][t][0] = sc->dt_sh[slot][t][0];
}

// Ghost columns of the HALO_LNS group from the mailbox of the step the fused
// tail just completed (it waited for every peer's flag): entry f of side s
// goes to ghost column ghostL - o[f] / ghostR + o[f] (grid-stride, one value
// per thread).
__global__ __launch_bounds__(BLOCK) void hf2d_p2p_unpack(ColList Lc, int ghostL, int ghostR, int ny, int cnt,
                                                        FusedX X) {
  const int par = (int)(*X.seq & 1);
  for (long t = (long)blockIdx.x * BLOCK + threadIdx.x; t < 2L * cnt; t += (long)gridDim.x * BLOCK) {
    const int side = t < cnt ? 0 : 1;
    if (!(X.sides & (1 << side))) continue;
    const int tt = (int)(t - (long)side * cnt), f = tt / ny, j = tt - f * ny;
    const real v = p2p_load(X.my_recv + ((long)par * 2 + side) * X.cap + tt);
    Lc.f[f][(long)(side == 0 ? ghostL - Lc.o[f] : ghostR + Lc.o[f]) * ny + j] = v;
  }
}
// register budget of OCC waves per SIMD (DeviceSolver::lns_occ, measured)
template <bool RES, int MODE, int OCC, int TURB = 2>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(OCC))) void hf2d_lns_step_occ(
    StepParams P, LnsArrays a, LeanTile T, DevScalars* sc, int slot, int slot_next, int serial,
    ResidualPack* partials, int part) {
  lns_step_body<RES, MODE, TURB>(P, a, T, sc, slot, slot_next, serial, partials, part);
}

// ---------------------------------------------------------------------------
// Lean mechanism-mode step (lean_mech.hpp): hf2d_lnm_step per 16 x 16 tile,
// then the kinetics of the listed cells and hf2d_lnm_hot.
// ---------------------------------------------------------------------------
// G_m of global cell (gi, gj) at tile coordinates (ii, jj): flow S / A / B
// and species A / B into the LDS planes that cell feeds.  dt_fill: the dt of
// the step the split fill F_m belongs to (SST's point-implicit destruction).
template <int TURB>
__device__ __forceinline__ void lnm_fill(StepParams& P, const LnmArrays& a, const LnmLayout& L, real* lds, int gi,
                                         int gj, int ii, int jj, CellLocal& c, real* mY, bool* early, bool* filled) {
  LnmFillIO<TURB> io(a, gi, gj, P.nx, P.ny);
  io.lds = lds;
  io.L = &L;
  io.aoff = L.a_at(ii, jj);
  io.boff = L.b_at(ii, jj);
  real mgx[1], mgy[1];
  int dummy = 0;
  (void)fill_compute<SK_MECH, LNM_NSB, LnmFillIO<TURB>, true>(P, io, c, mY, mgx, mgy, a.mech, a.nsp, gi, gj, true,
                                                               &dummy, early, filled);
  const int sC = L.s_at(ii, jj), aC = io.aoff, bC = io.boff;
  const bool zero = *early || !*filled;
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const int k = Lns<SK_SGT>::eqk(q);
    lds[L.oS + q * L.NC + sC] = c.S[k];
    if (aC >= 0) lds[L.oA + q * L.NA + aC] = zero ? 0.0 : c.A[k];
    if (bC >= 0) lds[L.oB + q * L.NB + bC] = zero ? 0.0 : c.B[k];
  }
  if (zero)   // (a skipped node stops the lean path; a solid one is never a neighbour)
    for (int t = 0; t < L.nspt; t++) {
      if (aC >= 0) lds[L.osA + t * L.NA + aC] = 0.0;
      if (bC >= 0) lds[L.osB + t * L.NB + bC] = 0.0;
    }
}

// STRIP: the strip has a right neighbour, so a partial last tile may hold its
// first ghost column (pass 1 below); without it the fill runs in one pass
// (56 instead of 112 B/lane of scratch for the SST kernel)
template <bool RES, int TURB, bool STRIP = true>
__device__ __forceinline__ void lnm_step_body(StepParams& P, const LnmArrays& a, const LeanTile& T, DevScalars* sc,
                                              int slot, int slot_next, int serial, ResidualPack* partials) {
  extern __shared__ real lds[];
  const unsigned b = a.lg ? tile_edge_first(xcd_remap(blockIdx.x, gridDim.x), T)
                          : tile_of_part(xcd_remap(blockIdx.x, gridDim.x), a.part, T);
  const LnmLayout L(T.TI, T.TJ, a.nsp - 1);
  // phase trace: wavefront 0 (slots 0..8) and the last wavefront (9, 10) of the workgroup
  unsigned long long* tr = a.tr ? a.tr + (long)b * 12 : nullptr;
  const bool tr0 = tr && threadIdx.x == 0, trl = tr && threadIdx.x == BLOCK - WAVE;
  if (tr0) tr[0] = rt_clock();
  // G_m runs with the dt of the step the split fill F_m belongs to; this
  // step's dt, scenario values and dt/dx, dt/dy are read up front as well (a
  // second read of the device scalars after the fills doubled the lean N-S
  // kernel's time)
  apply_dt(P, sc, slot);
  const real dt_now = P.dt;
  P.dt = sc->dt_val[slot_reset(slot)];
  const real dt_step = dt_cur(P, sc, slot);
  if (b == 0 && threadIdx.x == 0) {
    dt_reset(sc, slot_reset(slot));
    lag_head(P, sc, slot, slot_next);
    sc->dt_bits[slot] = d_to_bits(dt_step);   // folded (the kinetics read the word)
    sc->time_part += dt_step;
    sc->dt_val[slot] = dt_step;
    sc->hot_cnt[slot_next] = 0;
    // the interior tiles' list of a comm-overlap step (a later launch of this
    // step) starts empty whatever ran before (split steps reset hot_cnt only)
    sc->hot_cnt2[slot] = 0;
    scenario_next(P, sc, slot, slot_next);
  }
  int i, j, c, i0, j0;
  const bool mine = lean_tile_cell(P, T, (int)b, (int)threadIdx.x, &i, &j, &c, &i0, &j0);
  const int ii = (int)threadIdx.x / T.TJ, jj = (int)threadIdx.x - ii * T.TJ;
  int skip = 0;
  // 0. the previous step's halo from the mailbox into the ghost columns
  if (a.lg) {
    const FusedX& X = *a.xg;
    const unsigned long long seq_prev = *X.seq;
    if (seq_prev > 0 && !(X.skip & 4)) fx_ghost_prologue(P, X, a.lg, i0, j0, T.TI, T.TJ, seq_prev);
  }
  // 1a. ring cells: S, A or B only (on the threads after the tile's cells when
  // they fit in the workgroup, else on the first ones as a second fill)
  const int nring = 2 * (T.TI + T.TJ), own = T.TI * T.TJ;
  const int rbase = own + nring <= BLOCK ? own : 0;
  const int rt = (int)threadIdx.x - rbase;
  // 1a'. a strip's first ghost column inside a partial last tile (see lns).
  // Both fills go through one call site: a second inlined copy of the fill
  // pushed the SST kernel from 56 to 784 B/lane of scratch (2x slower).
#pragma unroll 1
  for (int pass = 0; pass < (STRIP ? 2 : 1); pass++) {
    int gi = -1, gj = 0, ri = 0, rj = 0;
    if (pass == 0) {
      if (rt >= 0 && rt < nring) {
        lns_ring_cell(T, rt, &ri, &rj);
        gi = i0 + ri;
        gj = j0 + rj;
      }
    } else if (!mine && (int)threadIdx.x < T.TIh * T.TJ && i == P.i1 && i < P.nx && j < P.ny) {
      gi = i;
      gj = j;
      ri = ii;
      rj = jj;
    }
    if (gi >= 0 && gi < P.nx && gj >= 0 && gj < P.ny) {
      CellLocal rc;
      real mY[LNM_NSB];
      bool early, filled;
      lnm_fill<TURB>(P, a, L, lds, gi, gj, ri, rj, rc, mY, &early, &filled);
    }
    if (pass == 0 && tr0) tr[1] = rt_clock();
  }
  // 1b. own cell: G_m, its level-m outputs, kept values for 2. and 3.
  LnmLevel lv;
  u64 CT = 0;
  uint8_t gf = 0, nbm = 0;
  bool early = true;
  const long N = a.N;
  const long idx = (long)i * P.ny + j;
  real bpre[6];
  if (mine) {
#pragma unroll
    for (int q = 0; q < 6; q++) bpre[q] = a.beta[Lns<SK_SGT>::eqk(q) * N + idx];
    CellLocal oc;
    real mY[LNM_NSB];
    bool filled = false;
    lnm_fill<TURB>(P, a, L, lds, i, j, ii, jj, oc, mY, &early, &filled);
    CT = oc.CT;
    gf = a.gf[idx];
    nbm = a.nb[idx];
    if (!early) {
      if (!filled) skip = 1;
      // mixture transport at T^m (fill_compute's tail: active nodes with a valid T)
      real mu = oc.mu, lam = oc.lam;
      if (is_active(CT) && !(oc.Tg < 0. || !(oc.Tg > MECH_TMIN))) mech_transport<LNM_NSB>(*a.mech, mY, oc.Tg, &mu, &lam);
      a.Uo[idx] = oc.U;
      a.Vo[idx] = oc.V;
      a.To[idx] = oc.Tg;
      a.muo[idx] = mu;
      a.lamo[idx] = lam;
      a.mu_to[idx] = oc.mu_t;
      if (TURB) {
        a.Src[(long)I_K * N + idx] = oc.Src[I_K];
        a.Src[(long)I_EPS * N + idx] = oc.Src[I_EPS];
      }
      if (gf & GF_SRCADD)
#pragma unroll
        for (int q = 0; q < 6; q++) {
          const int k = Lns<SK_SGT>::eqk(q);
          a.SrcAdd[k * N + idx] = oc.SrcAdd[k];
        }
      lv.U = oc.U;
      lv.V = oc.V;
      lv.Tg = oc.Tg;
      lv.k = oc.k;
      lv.BGX = oc.BGX;
      lv.BGY = oc.BGY;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const int k = Lns<SK_SGT>::eqk(q);
        lv.SrcAdd[q] = oc.SrcAdd[k];
        lv.F[q] = oc.F[k];
        lv.Src[q] = oc.Src[k];
      }
    }
  }
  if (tr0) tr[2] = rt_clock();
  if (trl) tr[9] = rt_clock();
  // species inputs of the predictor, loaded before the barrier (in flight
  // while the other wavefronts finish their fills)
  const int n1 = (nbm & NB_XL) ? 1 : 0, n2 = (nbm & NB_XR) ? 1 : 0;
  const int n3 = (nbm & NB_YU) ? 1 : 0, n4 = (nbm & NB_YD) ? 1 : 0;
  const long iL = (long)(i - n1) * P.ny + j, iR = (long)(i + n2) * P.ny + j, iU = idx + n3, iD = idx - n4;
  real ys0[LNM_NSB], ysL[LNM_NSB], ysR[LNM_NSB], ysU[LNM_NSB], ysD[LNM_NSB], bts[LNM_NSB];
  if (mine) {
#pragma unroll
    for (int s = 0; s < LNM_NSB; s++) {
      const long o = (long)(s < a.nsp ? s : a.nsp - 1) * N;
      ys0[s] = a.Ys[o + idx];
      ysL[s] = a.Ys[o + iL];
      ysR[s] = a.Ys[o + iR];
      ysU[s] = a.Ys[o + iU];
      ysD[s] = a.Ys[o + iD];
      bts[s] = a.betas[o + idx];
    }
  }
  P.dt = dt_now;   // this step's dt for the predictor and E_{m+1}
  __syncthreads();
  if (tr0) tr[3] = rt_clock();
  // 2. predict_m, flow and turbulence equations
  ResidualPack r;
  if (RES) {
    residual_reset(r);
#pragma unroll
    for (int k = 0; k < NEQ; k++) r.eq[k].i = r.eq[k].j = -1;
  }
  real dtl = 1.0;
  int neg = 0;
  const int nsp = a.nsp, bath = a.bath;
  if (mine) {
    const int sC = L.s_at(ii, jj), aC = L.a_at(ii, jj), bC = L.b_at(ii, jj);
    LnmPredictIO io{a, lds, L, lv, bpre, N, idx, idx, idx, idx, idx, sC, sC, sC, sC, sC, aC, aC, bC, bC, gf, {}};
    const bool act = is_active(CT);
    const u64 TT = a.TT[idx];
    if (!act) {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const int k = Lns<SK_SGT>::eqk(q);
        io.sn[k] = io.S(k);
        io.keep_dS(k);
      }
    } else {
      io.iL = iL;
      io.iR = iR;
      io.iU = iU;
      io.iD = iD;
      io.sL = sC - n1 * (T.TJ + 2);
      io.sR = sC + n2 * (T.TJ + 2);
      io.sU = sC + n3;
      io.sD = sC - n4;
      io.aL = aC - n1 * T.TJ;
      io.aR = aC + n2 * T.TJ;
      io.bU = bC + n3;
      io.bD = bC - n4;
      predict_core<RES>(P, io, CT, TT, n1, n2, n3, n4, P.gx0 + i, j, r);
    }
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const int k = Lns<SK_SGT>::eqk(q);
      a.Sp_out[k * N + idx] = io.sn[k];
    }
    if (tr0) tr[4] = rt_clock();
    // 3. species: transported ones by the predictor, the bath gas as the
    // remainder of the new rho (predict_cell_t order)
    real ysn[LNM_NSB];
    real sum = 0.0;
    const real rho_c = io.S(I_RHO);
#pragma unroll
    for (int s = 0; s < LNM_NSB; s++) {
      ysn[s] = 0.0;
      if (s < nsp && (s != bath || !act)) {
        const long o = (long)s * N;
        LnmSpeciesIO sio{a, lds, L, N, idx, iL, iR, iU, iD, o, s < bath ? s : s - 1, io.aL, io.aR, io.bU, io.bD, bC,
                         gf, ys0[s], ysL[s], ysR[s], ysU[s], ysD[s], bts[s], lv.SrcAdd[0], rho_c, 0.0};
        if (!act) {
          sio.out = sio.ys;
          a.Ys_out[o + idx] = sio.ys;
          sio.keep_dS(0);
        } else {
          predict_core<RES>(P, sio, CT, TT, n1, n2, n3, n4, P.gx0 + i, j, r);
          sum += sio.out;
        }
        ysn[s] = sio.out;
      }
    }
    if (act)
#pragma unroll
      for (int s = 0; s < LNM_NSB; s++)
        if (s == bath) {
          ysn[s] = io.sn[I_RHO] - sum;
          a.Ys_out[(long)s * N + idx] = ysn[s];
        }
    if (tr0) tr[5] = rt_clock();
    // 4. E_{m+1} of the new state, unless the kinetics change it (then hf2d_lnm_hot)
    if (!early) {
      const bool hot = act && io.sn[I_RHO] > 0.0 && lv.Tg >= a.mech->Tchem && P.dt > 0.0;
      const unsigned long long ball = __ballot(hot);
      if (ball) {
        const int lane = threadIdx.x & (WAVE - 1);
        const int leader = __ffsll((long long)ball) - 1;
        unsigned base = 0;
        if (lane == leader) base = atomicAdd(a.hot_n, (unsigned)__popcll(ball));
        base = __shfl(base, leader, WAVE);
        if (hot) a.hot[base + __popcll(ball & ((1ull << lane) - 1ull))] = (int)idx;
      }
      if (!hot) {
        const real S4[4] = {io.sn[0], io.sn[1], io.sn[2], io.sn[3]};
        LnmState st;
        if (!mech_state_node(P, *a.mech, nsp, S4, ysn, lv.U, lv.V, lv.Tg, lv.k, CT, lv.BGX, lv.BGY, &st, &dtl, &neg))
          skip = 1;
        a.Tso[idx] = st.T;
        a.pso[idx] = st.p;
        a.CPso[idx] = st.CP;
        a.kso[idx] = st.k;
      }
    }
  }
  if (tr0) tr[6] = rt_clock();
  if (trl) tr[10] = rt_clock();
  if (RES) {
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) shfl_merge(r, off);
    if ((threadIdx.x & (WAVE - 1)) == 0) partials[(long)b * (BLOCK / WAVE) + threadIdx.x / WAVE] = r;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  if (skip) atomicOr(&sc->neg_T, LNS_SKIP_ERR);
  __syncthreads();
  if (threadIdx.x == 0) {
    double mn = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) mn = fmin(mn, sdt[q]);
    if (serial) mn = fmin(mn, P.dt);
    dt_min(sc, slot_next, mn);
  }
  if (tr0) {
    tr[7] = rt_clock();
    tr[8] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID: wave/SIMD/CU/SE
    tr[11] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
}

// (two workgroups per CU: the LDS of a 16 x 16 tile is ~80 KB, so a budget
// of 2 waves per SIMD costs no occupancy)
template <bool RES, int TURB, bool STRIP = true>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(2))) void hf2d_lnm_step(
    StepParams P, LnmArrays a, LeanTile T, DevScalars* sc, int slot, int slot_next, int serial,
    ResidualPack* partials) {
  lnm_step_body<RES, TURB, STRIP>(P, a, T, sc, slot, slot_next, serial, partials);
}

// E_{m+1} of the cells the kinetics changed (after them): state and dt.
__global__ __launch_bounds__(BLOCK) void hf2d_lnm_hot(StepParams P, LnmArrays a, DevScalars* sc, int slot,
                                                       int slot_next, int serial) {
  apply_dt(P, sc, slot);
  const unsigned n = *a.hot_n;
  const long N = a.N;
  real dtl = 1.0;
  int neg = 0, skip = 0;
  for (unsigned q = blockIdx.x * BLOCK + threadIdx.x; q < n; q += gridDim.x * BLOCK) {
    const long idx = a.hot[q];
    real S4[4], ys[LNM_NSB];
#pragma unroll
    for (int k = 0; k < 4; k++) S4[k] = a.Sp_out[k * N + idx];
#pragma unroll
    for (int s = 0; s < LNM_NSB; s++) ys[s] = a.Ys_out[(long)(s < a.nsp ? s : a.nsp - 1) * N + idx];
    LnmState st;
    real d = 1.0;
    if (!mech_state_node(P, *a.mech, a.nsp, S4, ys, a.Uo[idx], a.Vo[idx], a.To[idx], a.ksi[idx], a.CT[idx],
                         a.BGX[idx], a.BGY[idx], &st, &d, &neg))
      skip = 1;
    dtl = fmin(dtl, d);
    a.Tso[idx] = st.T;
    a.pso[idx] = st.p;
    a.CPso[idx] = st.CP;
    a.kso[idx] = st.k;
  }
  for (int off = 1; off < WAVE; off <<= 1) dtl = fmin(dtl, __shfl_xor(dtl, off, WAVE));
  __shared__ double sdt[BLOCK / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) sdt[threadIdx.x / WAVE] = dtl;
  if (neg) atomicOr(&sc->neg_T, 1);
  if (skip) atomicOr(&sc->neg_T, LNS_SKIP_ERR);
  __syncthreads();
  if (threadIdx.x == 0) {
    double mn = sdt[0];
    for (int q = 1; q < BLOCK / WAVE; q++) mn = fmin(mn, sdt[q]);
    if (serial) mn = fmin(mn, P.dt);
    if (mn < 1.0) dt_min(sc, slot_next, mn);
  }
}

__global__ __launch_bounds__(BLOCK) void hf2d_wall_solid(StepParams P, SoA s, real* qdir, long c0, long c1) {
  const long c = c0 + (long)blockIdx.x * BLOCK + threadIdx.x;
  if (c >= c1) return;
  const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
  wall_heat_solid_cell(P, s, qdir, i, j);
}

__global__ __launch_bounds__(BLOCK) void hf2d_wall_wall(StepParams P, SoA s, const real* qdir, long c0, long c1,
                                                         const DevScalars* sc, int slot) {
  apply_dt(P, sc, slot);
  const long c = c0 + (long)blockIdx.x * BLOCK + threadIdx.x;
  if (c >= c1) return;
  const int i = (int)(c / P.ny), j = (int)(c - (long)i * P.ny);
  wall_heat_wall_cell(P, s, qdir, i, j);
}

// K10 in two passes: friction velocity of the wall nodes this strip owns
// (merged over the strips on the host), then y+ of every owned cell
__global__ __launch_bounds__(BLOCK) void hf2d_wall_uw(SoA s, const long* own, int n, real* uw, uint8_t* ok) {
  const int k = blockIdx.x * BLOCK + threadIdx.x;
  if (k >= n) return;
  const long w = own[k];
  const bool g = is_wall_gas(s.CT[w]);
  ok[k] = g ? 1 : 0;
  uw[k] = g ? wall_friction_velocity(s, w) : 0.;
}
__global__ __launch_bounds__(BLOCK) void hf2d_yplus(SoA s, long c0, long c1, const real* uw, const uint8_t* ok) {
  const long c = c0 + (long)blockIdx.x * BLOCK + threadIdx.x;
  if (c >= c1) return;
  y_plus_apply(s, c, uw, ok);
}


__global__ void hf2d_pack(ColList L, int col, int ny, real* buf) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L.nf * ny) return;
  const int f = t / ny, j = t - f * ny;
  buf[t] = L.f[f][(long)col * ny + j];
}
__global__ void hf2d_unpack(ColList L, int col, int ny, const real* buf) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L.nf * ny) return;
  const int f = t / ny, j = t - f * ny;
  L.f[f][(long)col * ny + j] = buf[t];
}
// Both sides in one launch (sides: bit 0 left, bit 1 right).
// dt slot's shards into its word (before a host transport sends the word)
__global__ void hf2d_dt_commit(DevScalars* sc, int slot) {
  if (threadIdx.x == 0) sc->dt_bits[slot] = d_to_bits(dt_get(sc, slot));
}
// MIN of the peers' dt into this rank's slot (exchange_dt, in-process group)
__global__ void hf2d_fold_dt(DevScalars* sc, int slot, const double* dt_recv, int nranks, int rank) {
  if (threadIdx.x != 0) return;
  double m = dt_get(sc, slot);
  for (int q = 0; q < nranks; q++)
    if (q != rank) m = fmin(m, dt_recv[q]);
  sc->dt_bits[slot] = d_to_bits(m);
}

// (dslot >= 0: also commits that dt slot's shards into its word, which the
// host transports send)
__global__ void hf2d_pack2(ColList L, int colL, int colR, int ny, real* bufL, real* bufR, int sides,
                           DevScalars* sc, int dslot) {
  const int cnt = L.nf * ny;
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0 && dslot >= 0) sc->dt_bits[dslot] = d_to_bits(dt_get(sc, dslot));
  const bool right = t >= cnt;
  if (right) t -= cnt;
  if (t >= cnt || !(sides & (right ? 2 : 1))) return;
  const int f = t / ny, j = t - f * ny;
  (right ? bufR : bufL)[t] = L.f[f][(long)(right ? colR - L.o[f] : colL + L.o[f]) * ny + j];
}
// Also folds the dt gathered from the other ranks (ndt > 0: dtr[q], q != self)
// into the next dt slot: MIN of positive doubles, exact in any order.
__global__ void hf2d_unpack2(ColList L, int colL, int colR, int ny, const real* bufL, const real* bufR,
                             int sides, DevScalars* sc, int dslot, const double* dtr, int ndt, int self) {
  const int cnt = L.nf * ny;
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0 && ndt > 0) {
    double m = dt_get(sc, dslot);
    for (int q = 0; q < ndt; q++)
      if (q != self) m = fmin(m, dtr[q]);
    sc->dt_bits[dslot] = d_to_bits(m);
  }
  const bool right = t >= cnt;
  if (right) t -= cnt;
  if (t >= cnt || !(sides & (right ? 2 : 1))) return;
  const int f = t / ny, j = t - f * ny;
  L.f[f][(long)(right ? colR + L.o[f] : colL - L.o[f]) * ny + j] = (right ? bufR : bufL)[t];
}

// ---------------------------------------------------------------------------
// xGMI peer-to-peer halo transport (default for multi-GPU strips).
//
// Every rank owns one fine-grained "mailbox" allocation, mapped into its
// peers with IPC handles:
//   flags[nranks]  u64   step sequence number last published by rank q
//   dtr[2][nranks] f64   dt of rank q for sequence parity 0/1
//   recv[2][2][cap] f64  halo columns for parity 0/1 from the left/right
// One single-workgroup kernel per exchange replaces pack + RCCL group +
// unpack: it stores this rank's boundary columns straight into the
// neighbours' mailboxes and its dt into every peer's, publishes its flag,
// waits (bounded) for every peer's flag of the same sequence number, then
// unpacks its own mailbox into the ghost columns and folds the MIN of all dt
// into the next dt slot -- bitwise the RCCL path's result.
// Ordering without system-scope fences: mailbox data and flags are written
// with system-coherent stores (p2p_store: they bypass the non-coherent L2),
// and a wave's stores are complete (s_waitcnt vmcnt(0)) before any flag is
// stored; a reader issues its system-coherent data loads only after it has
// seen the flag.  A __threadfence_system() would also write back the whole
// L2 of the XCD (buffer_wbl2), which cost ~3 us per step in the fused kernel.
// Parity double buffering is safe without a second handshake: a peer writes
// parity p again only at sequence s+2, after it has seen this rank's flag
// s+1, which is published after the unpack of s.  The sequence counter lives
// in device memory, so the kernel replays unchanged inside step graphs.
// ---------------------------------------------------------------------------


struct P2PArgs {
  ColList L;
  int first, last, ghostL, ghostR, ny, cnt, sides;
  long cap;                              // doubles per (parity, side) mailbox slot
  real* peer_recv_l;                     // left neighbour's recv base (this rank is its right side)
  real* peer_recv_r;                     // right neighbour's recv base
  real* my_recv;
  unsigned long long* const* peer_flags; // [nranks] flag array of each rank (self: own)
  double* const* peer_dtr;               // [nranks] dtr array of each rank
  unsigned long long* my_flags;
  double* my_dtr;
  unsigned long long* seq;               // device-side sequence counter
  DevScalars* sc;
  int dslot, fold_dt, rank, nranks;
};



__global__ __launch_bounds__(P2P_THREADS) void hf2d_p2p_xchg(P2PArgs a) {
  const unsigned long long seq = *a.seq + 1;
  const int par = (int)(seq & 1);
  const int ny = a.ny;
  // 1. push boundary columns and this rank's dt into the peers' mailboxes:
  // PER loads of a thread in flight, then its PER system-coherent stores (one
  // load latency per batch instead of one per value: the N-S halo is 23-43
  // fields x ny per side)
  constexpr int PER = 16;
  const int total = ((a.sides & 1) ? a.cnt : 0) + ((a.sides & 2) ? a.cnt : 0);
  for (int base = 0; base < total; base += PER * P2P_THREADS) {
    real v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int t = base + u * P2P_THREADS + threadIdx.x;
      if (t < total) {
        const bool right = !(a.sides & 1) || t >= a.cnt;
        const int tt = (a.sides & 1) && right ? t - a.cnt : t;
        const int f = tt / ny, j = tt - f * ny;
        v[u] = a.L.f[f][(long)(right ? a.last - a.L.o[f] : a.first + a.L.o[f]) * ny + j];
      }
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int t = base + u * P2P_THREADS + threadIdx.x;
      if (t < total) {
        const bool right = !(a.sides & 1) || t >= a.cnt;
        const int tt = (a.sides & 1) && right ? t - a.cnt : t;
        // the left neighbour receives "from right", the right one "from left"
        real* dst = right ? a.peer_recv_r + ((long)par * 2) * a.cap : a.peer_recv_l + ((long)par * 2 + 1) * a.cap;
        p2p_store(dst + tt, v[u]);
      }
    }
  }
  const double mydt = dt_get(a.sc, a.dslot);
  for (int q = threadIdx.x; q < a.nranks; q += P2P_THREADS)
    if (q != a.rank) p2p_store(a.peer_dtr[q] + par * a.nranks + a.rank, mydt);
  // system-coherent stores drained (vmcnt) in every wave before the flag:
  // no L2 writeback needed, nothing of this kernel sits dirty in the L2
  vm_drain();
  __syncthreads();
  // 2. publish, 3. wait for every peer's publication of the same sequence
  for (int q = threadIdx.x; q < a.nranks; q += P2P_THREADS)
    if (q != a.rank) __hip_atomic_store(&a.peer_flags[q][a.rank], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const bool failed = __hip_atomic_load(&a.sc->neg_T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2;
  __shared__ double s_dt[P2P_THREADS];
  double dmin = mydt;   // each polling thread folds the dt of the peers it waited for
  for (int q = threadIdx.x; q < a.nranks; q += P2P_THREADS) {
    if (q == a.rank || failed) continue;   // after one timeout, stop waiting (the host reports it)
    long spins = 0;
    bool ok = true;
    while (__hip_atomic_load(&a.my_flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > P2P_SPIN_LIMIT) {
        atomicOr(&a.sc->neg_T, 2);
        ok = false;
        break;
      }
    }
    if (ok) (void)p2p_acquire(&a.my_flags[q]);   // order the mailbox reads after the flag
    if (ok) dmin = fmin(dmin, p2p_load(a.my_dtr + par * a.nranks + q));
  }
  s_dt[threadIdx.x] = dmin;
  __syncthreads();
  // 4. unpack this rank's mailbox into the ghost columns: all loads of a
  // thread first, then its stores (the stores may alias nothing the loads
  // read, but the compiler cannot know that)
  for (int base = 0; base < total; base += PER * P2P_THREADS) {
    real v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int t = base + u * P2P_THREADS + threadIdx.x;
      if (t < total) {
        const bool right = !(a.sides & 1) || t >= a.cnt;
        const int tt = (a.sides & 1) && right ? t - a.cnt : t;
        v[u] = p2p_load(a.my_recv + ((long)par * 2 + (right ? 1 : 0)) * a.cap + tt);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int t = base + u * P2P_THREADS + threadIdx.x;
      if (t < total) {
        const bool right = !(a.sides & 1) || t >= a.cnt;
        const int tt = (a.sides & 1) && right ? t - a.cnt : t;
        const int f = tt / ny, j = tt - f * ny;
        a.L.f[f][(long)(right ? a.ghostR + a.L.o[f] : a.ghostL - a.L.o[f]) * ny + j] = v[u];
      }
    }
  }
  // 5. global dt: MIN over ranks (exact in any order)
  if (threadIdx.x == 0) {
    if (a.fold_dt) {
      double m = mydt;
      for (int q = 0; q < a.nranks && q < P2P_THREADS; q++) m = fmin(m, s_dt[q]);
      a.sc->dt_bits[a.dslot] = d_to_bits(m);
    }
    *a.seq = seq;
  }
}

// ---------------------------------------------------------------------------
// DeviceSolver
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Kernel tables: the template variants a step can select, indexed by the
// selecting parameters (the host dispatch is a table lookup, not a ladder).
// ---------------------------------------------------------------------------
using PredictK = void (*)(StepParams, SoA, SoA, long, long, DevScalars*, int, int, int, ResidualPack*);
// [residual][SK_* mode]
static const PredictK kPredict[2][4] = {
    {hf2d_predict<false, SK_GENERIC>, hf2d_predict<false, SK_SGL>, hf2d_predict<false, SK_SGT>,
     hf2d_predict<false, SK_MECH>},
    {hf2d_predict<true, SK_GENERIC>, hf2d_predict<true, SK_SGL>, hf2d_predict<true, SK_SGT>,
     hf2d_predict<true, SK_MECH>}};

using FillK = void (*)(StepParams, SoA, SoA, SoA, long, long, DevScalars*, int, int, int, int);
// register-budget slot of a fill: compiler default, 2, 3, 4 waves per SIMD
inline int occ_slot(int occ) { return occ == 2 ? 1 : occ == 3 ? 2 : occ == 4 ? 3 : 0; }
// [SK_* mode][occ_slot] (mechanism: the 9-species block)
static const FillK kFill[4][4] = {
    {hf2d_fill<SK_GENERIC>, hf2d_fill<SK_GENERIC>, hf2d_fill<SK_GENERIC>, hf2d_fill<SK_GENERIC>},
    {hf2d_fill<SK_SGL, 1>, hf2d_fill_occ<SK_SGL, 1, 2>, hf2d_fill_occ<SK_SGL, 1, 3>, hf2d_fill_occ<SK_SGL, 1, 4>},
    {hf2d_fill<SK_SGT, 1>, hf2d_fill_occ<SK_SGT, 1, 2>, hf2d_fill_occ<SK_SGT, 1, 3>, hf2d_fill_occ<SK_SGT, 1, 4>},
    {hf2d_fill<SK_MECH, 9>, hf2d_fill_occ<SK_MECH, 9, 2>, hf2d_fill_occ<SK_MECH, 9, 3>, hf2d_fill_occ<SK_MECH, 9, 4>}};

using TileK = void (*)(StepParams, LeanSoA, LeanTile, DevScalars*, int, int, int, ResidualPack*, int);
using TileFxK = void (*)(StepParams, LeanSoA, LeanTile, DevScalars*, int, int, int, ResidualPack*, const FusedX*);
using TileTrK = void (*)(StepParams, LeanSoA, LeanTile, DevScalars*, int, int, int, ResidualPack*,
                         unsigned long long*);
// [single gas][cells per thread - 1][0 plain, 1 outputs, 2 residual]
static const TileK kTile[2][2][3] = {
    {{hf2d_lean_tile<false, false, false, 0, 1>, hf2d_lean_tile<false, true, false, 0, 1>,
      hf2d_lean_tile<true, true, false, 0, 1>},
     {hf2d_lean_tile<false, false, false, 0, 2>, hf2d_lean_tile<false, true, false, 0, 2>,
      hf2d_lean_tile<true, true, false, 0, 2>}},
    {{hf2d_lean_tile<false, false, true, 0, 1>, hf2d_lean_tile<false, true, true, 0, 1>,
      hf2d_lean_tile<true, true, true, 0, 1>},
     {hf2d_lean_tile<false, false, true, 0, 2>, hf2d_lean_tile<false, true, true, 0, 2>,
      hf2d_lean_tile<true, true, true, 0, 2>}}};
static const TileFxK kTileFx[2][2][3] = {
    {{hf2d_lean_tile_fx<false, false, false, 1>, hf2d_lean_tile_fx<false, true, false, 1>,
      hf2d_lean_tile_fx<true, true, false, 1>},
     {hf2d_lean_tile_fx<false, false, false, 2>, hf2d_lean_tile_fx<false, true, false, 2>,
      hf2d_lean_tile_fx<true, true, false, 2>}},
    {{hf2d_lean_tile_fx<false, false, true, 1>, hf2d_lean_tile_fx<false, true, true, 1>,
      hf2d_lean_tile_fx<true, true, true, 1>},
     {hf2d_lean_tile_fx<false, false, true, 2>, hf2d_lean_tile_fx<false, true, true, 2>,
      hf2d_lean_tile_fx<true, true, true, 2>}}};
static const TileTrK kTileTr[2][2] = {{hf2d_lean_tile_tr<false, 1>, hf2d_lean_tile_tr<false, 2>},
                                      {hf2d_lean_tile_tr<true, 1>, hf2d_lean_tile_tr<true, 2>}};
// single gas, small workgroups: [0: 128 threads, 1: 64][cells per thread - 1][variant]
#define HF2D_NT_ROW(K, NT, CPT) {K<false, false, NT, CPT>, K<false, true, NT, CPT>, K<true, true, NT, CPT>}
static const TileK kTileNt[2][2][3] = {{HF2D_NT_ROW(hf2d_lean_tile_nt, 128, 1), HF2D_NT_ROW(hf2d_lean_tile_nt, 128, 2)},
                                       {HF2D_NT_ROW(hf2d_lean_tile_nt, 64, 1), HF2D_NT_ROW(hf2d_lean_tile_nt, 64, 2)}};
static const TileFxK kTileFxNt[2][2][3] = {
    {HF2D_NT_ROW(hf2d_lean_tile_fx_nt, 128, 1), HF2D_NT_ROW(hf2d_lean_tile_fx_nt, 128, 2)},
    {HF2D_NT_ROW(hf2d_lean_tile_fx_nt, 64, 1), HF2D_NT_ROW(hf2d_lean_tile_fx_nt, 64, 2)}};
#undef HF2D_NT_ROW
static const TileTrK kTileTrNt[2][2] = {{hf2d_lean_tile_tr_nt<128, 1>, hf2d_lean_tile_tr_nt<128, 2>},
                                        {hf2d_lean_tile_tr_nt<64, 1>, hf2d_lean_tile_tr_nt<64, 2>}};
// threads per workgroup of the inviscid tile kernel: 256, or 128 / 64 (single gas)
inline int tile_nt(int want, bool sg) { return sg && (want == 128 || want == 64) ? want : BLOCK; }

using LeanEulerK = void (*)(StepParams, LeanSoA, long, long, DevScalars*, int, int, int, ResidualPack*);
// [residual][first lean step: from the generic arrays]
static const LeanEulerK kLeanEuler[2][2] = {{hf2d_lean_euler<false, false>, hf2d_lean_euler<false, true>},
                                            {hf2d_lean_euler<true, false>, hf2d_lean_euler<true, true>}};

using LnsK = void (*)(StepParams, LnsArrays, LeanTile, DevScalars*, int, int, int, ResidualPack*, int);
// [laminar, k-eps, SST, SA][residual][register budget: default, 3, 5 waves per SIMD]
static const LnsK kLns[4][2][3] = {
    {{hf2d_lns_step<false, SK_SGL>, hf2d_lns_step_occ<false, SK_SGL, 3>, hf2d_lns_step_occ<false, SK_SGL, 5>},
     {hf2d_lns_step<true, SK_SGL>, hf2d_lns_step<true, SK_SGL>, hf2d_lns_step<true, SK_SGL>}},
    {{hf2d_lns_step<false, SK_SGT>, hf2d_lns_step_occ<false, SK_SGT, 3>, hf2d_lns_step_occ<false, SK_SGT, 5>},
     {hf2d_lns_step<true, SK_SGT>, hf2d_lns_step<true, SK_SGT>, hf2d_lns_step<true, SK_SGT>}},
    {{hf2d_lns_step<false, SK_SGT, 3>, hf2d_lns_step_occ<false, SK_SGT, 3, 3>, hf2d_lns_step_occ<false, SK_SGT, 5, 3>},
     {hf2d_lns_step<true, SK_SGT, 3>, hf2d_lns_step<true, SK_SGT, 3>, hf2d_lns_step<true, SK_SGT, 3>}},
    {{hf2d_lns_step<false, SK_SGT, 4>, hf2d_lns_step_occ<false, SK_SGT, 3, 4>, hf2d_lns_step_occ<false, SK_SGT, 5, 4>},
     {hf2d_lns_step<true, SK_SGT, 4>, hf2d_lns_step<true, SK_SGT, 4>, hf2d_lns_step<true, SK_SGT, 4>}}};

using LnsFxK = void (*)(StepParams, LnsArrays, LeanTile, DevScalars*, int, int, int, ResidualPack*, FusedX, ColList,
                        const ColList*);
// [laminar, k-eps, SST, SA][residual] (the default kernels' register budgets)
static const LnsFxK kLnsFx[4][2] = {
    {hf2d_lns_step_fx<false, SK_SGL, 2>, hf2d_lns_step_fx<true, SK_SGL, 2>},
    {hf2d_lns_step_fx3<false, SK_SGT, 2>, hf2d_lns_step_fx<true, SK_SGT, 2>},
    {hf2d_lns_step_fx3<false, SK_SGT, 3>, hf2d_lns_step_fx<true, SK_SGT, 3>},
    {hf2d_lns_step_fx3<false, SK_SGT, 4>, hf2d_lns_step_fx<true, SK_SGT, 4>}};

struct DevBuf {
  std::vector<void*> ptrs;
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
    HIP_CHECK(hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(T)));
    ptrs.push_back(p);
    return (T*)p;
  }
  ~DevBuf() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

struct LocalHostComm : Comm {
  std::shared_ptr<LocalGroup> g;
  int r;
  LocalHostComm(std::shared_ptr<LocalGroup> g_, int r_) : g(std::move(g_)), r(r_) {}
  std::vector<std::string> allgather_bytes(const std::string& mine) override {
    g->blobs[r] = mine;
    g->barrier();
    std::vector<std::string> all(g->blobs.begin(), g->blobs.end());
    g->barrier();
    return all;
  }
  int rank() const override { return r; }
  int size() const override { return g->n; }
  real allreduce_min(real v) override { return g->reduce(r, v, 0); }
  real allreduce_sum(real v) override { return g->reduce(r, v, 1); }
  int allreduce_max_int(int v) override { return (int)g->reduce(r, (double)v, 2); }
  void allreduce_residual(ResidualPack& p) override {
    g->packs[r] = p;
    g->barrier();
    ResidualPack a = g->packs[0];
    for (int q = 1; q < g->n; q++) residual_merge_lex(a, g->packs[q]);
    g->barrier();
    p = a;
  }
};

std::shared_ptr<LocalGroup> make_local_group(int n) { return std::make_shared<LocalGroup>(n); }

struct DeviceSolver::Impl {
  DevBuf mem;
  hipStream_t stream = nullptr;
  // comm overlap: the halo of the edge tiles travels on comm_stream while the
  // interior tiles compute on `stream` (events ev_edge / ev_halo join them)
  hipStream_t comm_stream = nullptr;
  hipEvent_t ev_edge = nullptr, ev_halo = nullptr;
  // device arrays (same roles as HostArrays)
  real *S[2], *A[2], *B[2], *F, *Src, *SrcAdd, *beta, *dSdx[2], *dSdy[2];
  real *U[2], *V[2], *Tg[2], *p, *kk, *R, *CP, *lam, *mu, *mu_t, *lam_t, *Diff, *Y;
  real *l_min, *y_plus, *Re_local, *BGX, *BGY, *Tf, *Q_conv, *grad, *qdir;
  u64 *CT, *TT;
  uint8_t* nb;
  // lean inviscid state: pre-chemistry species and pressure (ping-pong with
  // U/V on pbuf), per-cell neighbour/publish byte
  real *Spre[2], *P2[2];
  // lean N-S: second level of CP / mu / lam / k (the first is the generic array)
  real *CP2 = nullptr, *mu2 = nullptr, *lam2 = nullptr, *kk2 = nullptr, *mu_t2 = nullptr;
  // lean mechanism step: second level of p and both levels of the stored T
  // (the thermodynamic state T, p, Cp, k of lean_mech.hpp; Cp / k share CP2 / kk2)
  real *p2 = nullptr, *Tst[2] = {nullptr, nullptr};
  unsigned long long* lnm_trace = nullptr;   // HF2D_LNM_TRACE phase clocks
  long lnm_trace_n = 0;
  uint8_t* lb;
  uint8_t* gf;   // generic-stepper GF_* traffic flags
  int32_t* wslot;
  // K10 (y+): owned wall nodes, their friction velocities, all strips' values
  long* wall_own = nullptr;
  real *wall_uw = nullptr, *uw_all = nullptr;
  uint8_t *wall_ok = nullptr, *uw_all_ok = nullptr;
  // mechanism mode (SK_MECH): species block, Ys ping-pongs with S (sbuf)
  MechData* mech = nullptr;
  int nsp = 0;
  std::unique_ptr<ChemMechPack> chem_pack;   // MFMA kinetics kernel's mechanism image
  int* chem_list = nullptr;                  // compacted kinetics: reacting cells of the step
  unsigned* chem_count = nullptr;
  real *Ys[2] = {nullptr, nullptr}, *As = nullptr, *Bs = nullptr, *Fs = nullptr, *betas = nullptr;
  real *dSdxs[2] = {nullptr, nullptr}, *dSdys[2] = {nullptr, nullptr};
  SpeciesProps* species = nullptr;
  ScenarioTables* scen = nullptr;
  long* probe_idx = nullptr;   // K8 monitor probes (sample_monitors)
  real* probe_out = nullptr;
  DevScalars* sc = nullptr;
  DevScalars* sc_host = nullptr;   // pinned
  bool sc_kernel = true;           // sync_scalars: hf2d_scalars_out instead of a copy (HF2D_SC_KERNEL=0: copy)
  // single GPU: the last (output) lean tile step of a host call wrote the
  // scalars into sc_host itself (DeviceSolver::host_tail); sync_scalars then
  // only waits
  bool sc_mirrored = false;
  unsigned* host_done = nullptr;   // host_tail's completion counters
  hipEvent_t lnm_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // DeviceSolver::lnm_timing
  FusedX* fx_dev = nullptr;   // fx_device: the tile kernels' copy of fused_args()
  FusedX fx_dev_host{};
  bool fx_dev_valid = false;
  // fused lean N-S / mechanism steps: the HALO_LNS list of the last fused
  // step, whose halo is still in the mailbox (lns_ghost_pending), and device
  // copies of the lists of both buffer parities (the next step's prologue)
  ColList lns_pend{};
  ColList* lc_dev = nullptr;
  ColList lc_host[2]{};
  bool lc_valid[2] = {false, false};
  int lc_next = 0;
  ResidualPack* partials = nullptr;
  ResidualPack* res_out = nullptr;
  ResidualPack* res_host = nullptr;   // pinned
  long max_partials = 0;
  real* halo_send[2] = {nullptr, nullptr};
  real* halo_recv[2] = {nullptr, nullptr};
  long halo_cap = 0;
  double* dt_recv = nullptr;   // dt of every rank (gathered with the halo)
  ncclComm_t comm = nullptr;
  std::shared_ptr<LocalGroup> local;   // in-process virtual ranks (testing)
  int rank = 0, nranks = 1;
  // xGMI peer-to-peer transport (hf2d_p2p_xchg)
  struct P2P {
    bool on = false;
    char* base = nullptr;                 // fine-grained mailbox (p2p_layout)
    size_t bytes = 0, off_dtr = 0, off_recv = 0;
    unsigned long long* seq = nullptr;    // device-side exchange counter
    unsigned* done = nullptr;             // fused tile kernel: finished workgroups
    std::vector<char*> peer_base;         // mailbox of every rank (self: base)
    std::vector<void*> opened;            // IPC mappings to close
    unsigned long long** d_flags = nullptr;
    double** d_dtr = nullptr;
    bool loop = false;                    // p2p_loopback: the neighbours' mailboxes are this rank's own
    // mailbox the edge pushes of `side` land in (0: the left neighbour's,
    // whose right side this rank is); loopback: this rank's own mailbox of
    // that side, so the ghost columns take the strip's own edge values
    real* push_base(int side, int rank, long cap) const {
      if (loop) return (real*)(base + off_recv) + (side == 0 ? -cap : cap);
      return (real*)(peer_base[side == 0 ? rank - 1 : rank + 1] + off_recv);
    }
  } p2p;

  LeanSoA lean_view(const HostArrays& h, int sb, int ab, int db, int pb, bool fromg) const {
    LeanSoA L;
    L.N = h.N;
    L.Sin = S[sb];
    L.Sout = S[1 - sb];
    L.Pin_s = Spre[pb];
    L.Pout_s = Spre[1 - pb];
    L.beta = beta;
    L.Uin = U[pb];
    L.Vin = V[pb];
    L.Pin = fromg ? p : P2[pb];
    L.Uout = U[1 - pb];
    L.Vout = V[1 - pb];
    L.Pout = P2[1 - pb];
    L.Tout = Tg[1 - pb];
    L.dSdx_in = dSdx[db];
    L.dSdy_in = dSdy[db];
    L.dSdx_out = dSdx[1 - db];
    L.dSdy_out = dSdy[1 - db];
    L.CT = CT;
    L.lb = lb;
    L.CP = CP;
    L.R = R;
    L.kk = kk;
    L.Y = Y;
    L.Tf = Tf;
    L.BGX = BGX;
    L.BGY = BGY;
    L.SrcAdd = SrcAdd;
    L.gA = A[ab];
    L.gB = B[ab];
    L.gF = F;
    return L;
  }

  // lean N-S kernel arguments: Sp^m in S[1-sb], level m-1 primitives in
  // U/V/Tg[1-pb] and CPx[1-cb]; K_m writes Sp^{m+1} into S[sb], level m into
  // U/V/Tg[pb] and CPx[cb] (CPx[0] = the generic arrays)
  LnsArrays lns_arrays(const HostArrays& h, int sb, int pb, int cb, int db, int ab) const {
    LnsArrays a;
    a.N = h.N;
    a.Sp = S[1 - sb];
    a.Sp_out = S[sb];
    a.beta = beta;
    a.Ui = U[1 - pb];
    a.Vi = V[1 - pb];
    a.Ti = Tg[1 - pb];
    a.Uo = U[pb];
    a.Vo = V[pb];
    a.To = Tg[pb];
    real* const cpx[2] = {CP, CP2};
    real* const mux[2] = {mu, mu2};
    real* const lamx[2] = {lam, lam2};
    real* const kkx[2] = {kk, kk2};
    a.CPi = cpx[1 - cb];
    a.mui = mux[1 - cb];
    a.lami = lamx[1 - cb];
    a.kki = kkx[1 - cb];
    a.CPo = cpx[cb];
    a.muo = mux[cb];
    a.lamo = lamx[cb];
    a.kko = kkx[cb];
    real* const mutx[2] = {mu_t, mu_t2};
    a.mu_ti = mutx[1 - cb];
    a.mu_to = mutx[cb];
    a.l_min = l_min;
    a.y_plus = y_plus;
    a.Src = Src;
    a.gA = A[ab];
    a.gB = B[ab];
    a.gF = F;
    a.R = R;
    a.BGX = BGX;
    a.BGY = BGY;
    a.grad = grad;
    a.SrcAdd = SrcAdd;
    a.dSdx_in = dSdx[db];
    a.dSdy_in = dSdy[db];
    a.dSdx_out = dSdx[1 - db];
    a.dSdy_out = dSdy[1 - db];
    a.CT = CT;
    a.TT = TT;
    a.nb = nb;
    a.gf = gf;
    return a;
  }

  // lean mechanism step arguments (lean_mech.hpp): Sp^m in S[1-sb], its
  // post-kinetics species in Ys[sb]; every two-level array is read at
  // [1 - cb] and written at [cb] (transport m-1 -> m, state m -> m+1)
  LnmArrays lnm_arrays(const HostArrays& h, int sb, int pb, int cb, int db, int ab) const {
    LnmArrays a;
    a.N = h.N;
    a.mech = mech;
    a.nsp = nsp;
    a.bath = h.mech ? h.mech->bath : 0;
    a.Sp = S[1 - sb];
    a.Sp_out = S[sb];
    a.Ys = Ys[sb];
    a.Ys_out = Ys[1 - sb];
    a.beta = beta;
    a.betas = betas;
    a.Ui = U[1 - pb];
    a.Vi = V[1 - pb];
    a.Ti = Tg[1 - pb];
    a.Uo = U[pb];
    a.Vo = V[pb];
    a.To = Tg[pb];
    real* const mux[2] = {mu, mu2};
    real* const lamx[2] = {lam, lam2};
    real* const mutx[2] = {mu_t, mu_t2};
    real* const cpx[2] = {CP, CP2};
    real* const kkx[2] = {kk, kk2};
    real* const px[2] = {p, p2};
    a.mui = mux[1 - cb];
    a.lami = lamx[1 - cb];
    a.mu_ti = mutx[1 - cb];
    a.muo = mux[cb];
    a.lamo = lamx[cb];
    a.mu_to = mutx[cb];
    a.Tsi = Tst[1 - cb];
    a.psi = px[1 - cb];
    a.CPsi = cpx[1 - cb];
    a.ksi = kkx[1 - cb];
    a.Tso = Tst[cb];
    a.pso = px[cb];
    a.CPso = cpx[cb];
    a.kso = kkx[cb];
    a.l_min = l_min;
    a.y_plus = y_plus;
    a.BGX = BGX;
    a.BGY = BGY;
    a.grad = grad;
    a.Src = Src;
    a.SrcAdd = SrcAdd;
    a.gA = A[ab];
    a.gB = B[ab];
    a.gF = F;
    a.dSdx_in = dSdx[db];
    a.dSdy_in = dSdy[db];
    a.dSdx_out = dSdx[1 - db];
    a.dSdy_out = dSdy[1 - db];
    a.dSdxs_in = dSdxs[db];
    a.dSdys_in = dSdys[db];
    a.dSdxs_out = dSdxs[1 - db];
    a.dSdys_out = dSdys[1 - db];
    a.CT = CT;
    a.TT = TT;
    a.nb = nb;
    a.gf = gf;
    a.hot = chem_list;
    return a;
  }

  SoA view(const HostArrays& h, int sb, int ab, int db, int pb) const {
    SoA s;
    s.nx = h.nx;
    s.ny = h.ny;
    s.N = h.N;
    s.S = S[sb];
    s.A = A[ab];
    s.B = B[ab];
    s.F = F;
    s.Src = Src;
    s.SrcAdd = SrcAdd;
    s.beta = beta;
    s.dSdx = dSdx[db];
    s.dSdy = dSdy[db];
    s.U = U[pb];
    s.V = V[pb];
    s.Tg = Tg[pb];
    s.p = p;
    s.kk = kk;
    s.R = R;
    s.CP = CP;
    s.lam = lam;
    s.mu = mu;
    s.mu_t = mu_t;
    s.lam_t = lam_t;
    s.Diff = Diff;
    s.Y = Y;
    s.l_min = l_min;
    s.y_plus = y_plus;
    s.Re_local = Re_local;
    s.BGX = BGX;
    s.BGY = BGY;
    s.Tf = Tf;
    s.Q_conv = Q_conv;
    s.grad = grad;
    s.CT = CT;
    s.TT = TT;
    s.nb = nb;
    s.gf = gf;
    s.wslot = wslot;
    mech_view(s, sb, db);
    return s;
  }
  void mech_view(SoA& s, int yb, int db) const {
    s.mech = mech;
    s.nsp = nsp;
    if (!mech) return;
    s.Ys = Ys[yb];
    s.As = As;
    s.Bs = Bs;
    s.Fs = Fs;
    s.betas = betas;
    s.dSdxs = dSdxs[db];
    s.dSdys = dSdys[db];
  }
};

static int g_device_count_cache = -1;

bool gpu_available() {
  if (g_device_count_cache < 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    g_device_count_cache = n;
  }
  return g_device_count_cache > 0;
}

DeviceSolver::DeviceSolver(Case& c, int device, int gi0_, int gi1_) : SolverBase(c), impl(new Impl) {
  if (!gpu_available()) throw std::runtime_error("no HIP device available");
  dev = device;
  HIP_CHECK(hipSetDevice(dev));
  HIP_CHECK(hipStreamCreateWithFlags(&impl->stream, hipStreamNonBlocking));
  {
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, dev));
    cu_count = prop.multiProcessorCount;
  }
  if (const char* e = std::getenv("HF2D_SPLIT_XCD")) split_xcd = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_SPLIT_XCD_MECH")) split_xcd_mech = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_MECH_LAZY")) mech_lazy = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_CHEM_KERNEL")) chem_kernel = std::atoi(e);   // 1 compiled 2 MFMA 3 generic 4 hiprtc
  if (const char* e = std::getenv("HF2D_GRAD_EVERY")) grad_every = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_LNM_TI")) lnm_ti = std::atoi(e);
  if (const char* e = std::getenv("HF2D_PUSH_PER")) push_per = std::atoi(e);
  if (const char* e = std::getenv("HF2D_STAGGER")) tile_stagger = std::atoi(e);
  if (const char* e = std::getenv("HF2D_SC_KERNEL")) impl->sc_kernel = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_HOST_TAIL")) host_tail = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_DT_READ")) dt_read_mode = std::atoi(e);
  if (const char* e = std::getenv("HF2D_SKIP_SAME")) tile_skip_same = std::string(e) != "0";
  if (const char* e = std::getenv("HF2D_GHOST_PROLOGUE")) lns_ghost_prologue = std::string(e) != "0";
  gi0 = gi0_;
  gi1 = gi1_ < 0 ? c.J.nx : gi1_;
  // ghost columns: N-S strips keep two (the lean N-S / mechanism tiles
  // evaluate the fill of the first ghost column, which reads the second);
  // the split kernels read one, the inviscid ones one
  const int G = c.cfg.ProblemType == SM_NS ? 2 : 1;
  const int lh = gi0 > 0 ? G : 0, rh = gi1 < c.J.nx ? G : 0;
  l_off = lh;
  h.allocate((gi1 - gi0) + lh + rh, c.J.ny);
  const long N = h.N;
  Impl& m = *impl;
  for (int b = 0; b < 2; b++) {
    m.S[b] = m.mem.alloc<real>(NEQ * N);
    m.A[b] = m.mem.alloc<real>(NEQ * N);
    m.B[b] = m.mem.alloc<real>(NEQ * N);
    m.dSdx[b] = m.mem.alloc<real>(NEQ * N);
    m.dSdy[b] = m.mem.alloc<real>(NEQ * N);
    m.U[b] = m.mem.alloc<real>(N);
    m.V[b] = m.mem.alloc<real>(N);
    m.Tg[b] = m.mem.alloc<real>(N);
    m.Spre[b] = m.mem.alloc<real>(NCOMP * N);
    m.P2[b] = m.mem.alloc<real>(N);
  }
  m.lb = m.mem.alloc<uint8_t>(N);
  m.gf = m.mem.alloc<uint8_t>(N);
  m.F = m.mem.alloc<real>(NEQ * N);
  m.Src = m.mem.alloc<real>(NEQ * N);
  m.SrcAdd = m.mem.alloc<real>(NEQ * N);
  m.beta = m.mem.alloc<real>(NEQ * N);
  m.p = m.mem.alloc<real>(N);
  m.kk = m.mem.alloc<real>(N);
  m.R = m.mem.alloc<real>(N);
  m.CP = m.mem.alloc<real>(N);
  m.lam = m.mem.alloc<real>(N);
  m.mu = m.mem.alloc<real>(N);
  m.mu_t = m.mem.alloc<real>(N);
  m.lam_t = m.mem.alloc<real>(N);
  m.Diff = m.mem.alloc<real>(N);
  m.Y = m.mem.alloc<real>(NSPEC * N);
  m.l_min = m.mem.alloc<real>(N);
  m.y_plus = m.mem.alloc<real>(N);
  m.Re_local = m.mem.alloc<real>(N);
  m.BGX = m.mem.alloc<real>(N);
  m.BGY = m.mem.alloc<real>(N);
  m.Tf = m.mem.alloc<real>(N);
  m.Q_conv = m.mem.alloc<real>(N);
  m.grad = m.mem.alloc<real>(NGRAD * N);
  m.qdir = m.mem.alloc<real>(4 * N);
  m.CT = m.mem.alloc<u64>(N);
  m.TT = m.mem.alloc<u64>(N);
  m.nb = m.mem.alloc<uint8_t>(N);
  m.wslot = m.mem.alloc<int32_t>(N);
  h.allocate_mech(c);
  if (h.mech) {
    m.nsp = h.nsp;
    const long n = (long)m.nsp * N;
    m.mech = m.mem.alloc<MechData>(1);
    for (int b = 0; b < 2; b++) m.Ys[b] = m.mem.alloc<real>(n);
    m.As = m.mem.alloc<real>(n);
    m.Bs = m.mem.alloc<real>(n);
    m.Fs = m.mem.alloc<real>(n);
    m.betas = m.mem.alloc<real>(n);
    if (!h.dSdxs[0].empty())
      for (int b = 0; b < 2; b++) {
        m.dSdxs[b] = m.mem.alloc<real>(n);
        m.dSdys[b] = m.mem.alloc<real>(n);
      }
  }
  m.species = m.mem.alloc<SpeciesProps>(1);
  m.scen = m.mem.alloc<ScenarioTables>(1);
  m.sc = m.mem.alloc<DevScalars>(1);
  HIP_CHECK(hipHostMalloc((void**)&m.sc_host, sizeof(DevScalars), hipHostMallocDefault));
  m.host_done = m.mem.alloc<unsigned>((DT_SHARDS + 1) * FX_DONE_STRIDE);
  {
    // any tile shape (lean_tj) covers >= LEAN_TILE_MIN_TJ cells per workgroup
    const long nb_tile = (long)(gi1 - gi0 + 1) * ((h.ny + LEAN_TILE_MIN_TJ - 1) / LEAN_TILE_MIN_TJ);
    m.max_partials = std::max((N + BLOCK - 1) / BLOCK, nb_tile) * (BLOCK / WAVE);
  }
  m.partials = m.mem.alloc<ResidualPack>(m.max_partials);
  m.res_out = m.mem.alloc<ResidualPack>(1);
  HIP_CHECK(hipHostMalloc((void**)&m.res_host, sizeof(ResidualPack), hipHostMallocDefault));
  m.halo_cap = (long)MAX_HALO_FIELDS * h.ny;
  for (int d = 0; d < 2; d++) {
    m.halo_send[d] = m.mem.alloc<real>(m.halo_cap);
    m.halo_recv[d] = m.mem.alloc<real>(m.halo_cap);
  }
  // hipMemset on device memory is asynchronous and runs on the null stream,
  // which does not order against the non-blocking solver stream: drain the
  // zero-fills before upload() copies the state in.
  HIP_CHECK(hipDeviceSynchronize());
  upload();
}

DeviceSolver::~DeviceSolver() {
  try {
    flush_pending();
  } catch (...) {
  }
  graph.reset();
  host_comm.reset();
  if (impl) {
    if (impl->stream) (void)hipStreamSynchronize(impl->stream);
    for (void* p : impl->p2p.opened) (void)hipIpcCloseMemHandle(p);
    if (impl->comm) ncclCommDestroy(impl->comm);
    if (impl->sc_host) (void)hipHostFree(impl->sc_host);
    if (impl->res_host) (void)hipHostFree(impl->res_host);
    if (impl->comm_stream) (void)hipStreamSynchronize(impl->comm_stream);
    if (impl->ev_edge) (void)hipEventDestroy(impl->ev_edge);
    if (impl->ev_halo) (void)hipEventDestroy(impl->ev_halo);
    for (hipEvent_t e : impl->lnm_ev)
      if (e) (void)hipEventDestroy(e);
    if (impl->comm_stream) (void)hipStreamDestroy(impl->comm_stream);
    if (impl->stream) (void)hipStreamDestroy(impl->stream);
  }
}

void* DeviceSolver::stream() const { return (void*)impl->stream; }

void DeviceSolver::upload() {
  flush_pending();
  HIP_CHECK(hipSetDevice(dev));
  h.from_field(cs.J, gi0 - l_off);
  h.wall_slots(cs, gi0 - l_off, gi0, gi1);
  Impl& m = *impl;
  hipStream_t st = m.stream;
  const long N = h.N;
  if (!m.wall_own) {   // K10 buffers (sizes fixed by the grid's wall nodes)
    m.wall_own = m.mem.alloc<long>(h.wall_own.size());
    m.wall_uw = m.mem.alloc<real>(h.wall_own.size());
    m.wall_ok = m.mem.alloc<uint8_t>(h.wall_own.size());
    m.uw_all = m.mem.alloc<real>(cs.wall_nodes.size());
    m.uw_all_ok = m.mem.alloc<uint8_t>(cs.wall_nodes.size());
  }
  if (!h.wall_own.empty())
    HIP_CHECK(hipMemcpyAsync(m.wall_own, h.wall_own.data(), h.wall_own.size() * sizeof(long), hipMemcpyHostToDevice, st));
  auto cp = [&](void* d, const void* s, size_t bytes) { HIP_CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyHostToDevice, st)); };
  const size_t EQB = NEQ * N * sizeof(real), SB = N * sizeof(real);
  for (int b = 0; b < 2; b++) {
    cp(m.S[b], h.S[0].data(), EQB);
    cp(m.A[b], h.A.data(), EQB);
    cp(m.B[b], h.B.data(), EQB);
    cp(m.dSdx[b], h.dSdx[0].data(), EQB);
    cp(m.dSdy[b], h.dSdy[0].data(), EQB);
    cp(m.U[b], h.U[0].data(), SB);
    cp(m.V[b], h.V[0].data(), SB);
    cp(m.Tg[b], h.Tg[0].data(), SB);
  }
  cp(m.F, h.F.data(), EQB);
  cp(m.Src, h.Src.data(), EQB);
  cp(m.SrcAdd, h.SrcAdd.data(), EQB);
  cp(m.beta, h.beta.data(), EQB);
  cp(m.p, h.p.data(), SB);
  cp(m.kk, h.kk.data(), SB);
  cp(m.R, h.R.data(), SB);
  cp(m.CP, h.CP.data(), SB);
  cp(m.lam, h.lam.data(), SB);
  cp(m.mu, h.mu.data(), SB);
  cp(m.mu_t, h.mu_t.data(), SB);
  cp(m.lam_t, h.lam_t.data(), SB);
  cp(m.Diff, h.Diff.data(), SB);
  cp(m.Y, h.Y.data(), NSPEC * SB);
  cp(m.l_min, h.l_min.data(), SB);
  cp(m.y_plus, h.y_plus.data(), SB);
  cp(m.Re_local, h.Re_local.data(), SB);
  cp(m.BGX, h.BGX.data(), SB);
  cp(m.BGY, h.BGY.data(), SB);
  cp(m.Tf, h.Tf.data(), SB);
  cp(m.Q_conv, h.Q_conv.data(), SB);
  cp(m.grad, h.grad.data(), NGRAD * SB);
  cp(m.CT, h.CT.data(), N * sizeof(u64));
  cp(m.TT, h.TT.data(), N * sizeof(u64));
  cp(m.nb, h.nb.data(), N);
  compute_generic_flags(cs, h, gi0 - l_off);
  cp(m.gf, h.gf.data(), N);
  chem_fast_ok = cs.cfg.mech_mode() && chem_fast_available(cs.cfg.mech->name) &&
                 mech_is_builtin(*cs.cfg.mech, cs.cfg.mech->name);
  chem_rtc_ok = false;
  chem_rtc_why.clear();
  if (cs.cfg.mech_mode() && (chem_kernel == 4 || (chem_kernel == 0 && !chem_fast_ok && chem_rtc)))
    chem_rtc_ok = chem_rtc_prepare(*cs.cfg.mech->data_ptr(), &chem_rtc_why);   // compile now, not in a step graph
  lean_ok = lean_eligible(cs, &lean_why);
  sk_mode = sk_eligible(cs, &sgl_why);
  sgl_ok = sk_mode != SK_GENERIC;
  {
    // lean N-S (lean_ns.hpp): laminar single gas, flat, adiabatic walls, no
    // volume sources, every non-solid node set (fluxes of skipped or unset
    // nodes are not recomputable), one strip (no 2-column halo)
    auto no = [&](const char* w) {
      lns_ok = false;
      lns_why = w;
    };
    lns_ok = true;
    lns_why.clear();
    // turbulence: one of k-eps (without Chien's model: it reads the previous
    // p), k-omega SST or Spalart-Allmaras, and no eddy-viscosity term in the
    // dt (the own-cell part of the next fill has no gradients)
    const u64 other_models = TCT_Prandtl_Model | TCT_Integral_Model | TCT_k_omega_Model | TCT_Baldwin_Lomax_Model |
                             TCT_nut_92_Model | TCT_Smagorinsky_Model;
    lns_turb = 2;
    u64 models = 0;
    if (sk_mode != SK_SGL && sk_mode != SK_SGT) no("not single-gas N-S");
    else if (!cs.cfg.isAdiabaticWall) no("wall heat transfer");
    else if (cs.cfg.WallBlendCells > 0) no("WallBlendCells (split path only)");
    else if ((gi0 > 0 && l_off < 2) || (gi1 < cs.J.nx && h.nx - l_off - (gi1 - gi0) < 2)) no("one ghost column");
    else if (sk_mode == SK_SGT && cs.cfg.ViscousCFL > 0) no("viscous CFL with eddy viscosity");
    else
      for (long q = 0; q < N && lns_ok; q++) {
        if (h.gf[q] & GF_SRC) no("volume sources");
        else if (!has_all(h.CT[q], CT_SOLID) && !has_all(h.CT[q], CT_NODE_IS_SET)) no("unset non-solid node");
        else if (h.TT[q] & other_models) no("turbulence model other than k-eps, SST or SA");
        else models |= h.TT[q] & (TCT_k_eps_Model | TCT_k_omega_SST_Model | TCT_Spalart_Allmaras_Model);
      }
    // one model per kernel (fill_node's turbulence set)
    if (lns_ok && models == TCT_k_omega_SST_Model) lns_turb = 3;
    else if (lns_ok && models == TCT_Spalart_Allmaras_Model) lns_turb = 4;
    else if (lns_ok && models != 0 && models != TCT_k_eps_Model) no("more than one turbulence model");
    else if (lns_ok && models == TCT_k_eps_Model && cs.cfg.TurbExtModel == TEM_k_eps_Chien) no("Chien k-eps");
    if (lns_ok && !m.CP2) {
      m.CP2 = m.mem.alloc<real>(N);
      m.mu2 = m.mem.alloc<real>(N);
      m.lam2 = m.mem.alloc<real>(N);
      m.kk2 = m.mem.alloc<real>(N);
      m.mu_t2 = m.mem.alloc<real>(N);
    }
    if (m.CP2) {
      cp(m.CP2, h.CP.data(), SB);
      cp(m.mu2, h.mu.data(), SB);
      cp(m.lam2, h.lam.data(), SB);
      cp(m.kk2, h.kk.data(), SB);
      cp(m.mu_t2, h.mu_t.data(), SB);
    }
    lns_prev_mu_t = -1;
    lns_state = 0;
    cbuf = 0;
  }
  {
    // lean mechanism step (lean_mech.hpp): N-S, laminar or k-omega SST only
    // (SA / k-eps read values of the previous level before the state), no
    // eddy-viscosity or viscous CFL term in the dt (the state part has no
    // gradients), adiabatic walls, no volume sources, every non-solid node
    // set, one strip, <= LNM_NSB species
    auto no = [&](const char* w) {
      lnm_ok = false;
      lnm_why = w;
    };
    lnm_ok = true;
    lnm_why.clear();
    lnm_turb = 0;
    const u64 other_models = TCT_Prandtl_Model | TCT_Integral_Model | TCT_Spalart_Allmaras_Model |
                             TCT_k_omega_Model | TCT_k_eps_Model | TCT_Baldwin_Lomax_Model | TCT_nut_92_Model |
                             TCT_Smagorinsky_Model;
    if (!h.mech) no("not mechanism mode");
    else if (cs.cfg.ProblemType != SM_NS) no("not Navier-Stokes");
    else if (m.nsp > LNM_NSB || m.nsp < 2) no("species count outside the kernel's block");
    else if (!cs.cfg.isAdiabaticWall) no("wall heat transfer");
    else if (cs.cfg.WallBlendCells > 0) no("WallBlendCells (split path only)");
    else if ((gi0 > 0 && l_off < 2) || (gi1 < cs.J.nx && h.nx - l_off - (gi1 - gi0) < 2)) no("one ghost column");
    else if (cs.cfg.ViscousCFL > 0) no("viscous CFL");
    else if (h.ny < LNM_TILE) no("grid lower than one tile");
    else
      for (long q = 0; q < N && lnm_ok; q++) {
        if (h.gf[q] & GF_SRC) no("volume sources");
        else if (!has_all(h.CT[q], CT_SOLID) && !has_all(h.CT[q], CT_NODE_IS_SET)) no("unset non-solid node");
        else if (h.TT[q] & other_models) no("turbulence model other than k-omega SST");
        else if (has_all(h.TT[q], TCT_k_omega_SST_Model)) lnm_turb = 3;
      }
    if (lnm_ok) {
      if (!m.CP2) {
        m.CP2 = m.mem.alloc<real>(N);
        m.mu2 = m.mem.alloc<real>(N);
        m.lam2 = m.mem.alloc<real>(N);
        m.kk2 = m.mem.alloc<real>(N);
        m.mu_t2 = m.mem.alloc<real>(N);
      }
      if (!m.p2) {
        m.p2 = m.mem.alloc<real>(N);
        m.Tst[0] = m.mem.alloc<real>(N);
        m.Tst[1] = m.mem.alloc<real>(N);
      }
      if (!m.chem_list) {
        m.chem_list = m.mem.alloc<int>(N);
        m.chem_count = m.mem.alloc<unsigned>(1);
      }
    }
  }
  lean_sg_ok = lean_ok && lean_single_gas(cs);
  any_cauchy_x = lean_any_cauchy_x(cs);
  lean_has_cauchy_x = lean_ok && any_cauchy_x;
  ghost_mode = -1;
  if (lean_ok) {
    lean_bytes = lean_flags(h, cs.cfg.ProblemType);
    if (!lean_plain)
      for (auto& b : lean_bytes) b &= (uint8_t)~LB_PLAIN;
    cp(m.lb, lean_bytes.data(), N);
  }
  lean_state = 0;
  cp(m.wslot, h.wslot.data(), N * sizeof(int32_t));
  cp(m.species, &cs.cfg.species, sizeof(SpeciesProps));
  if (h.mech) {
    h.mech_from_case(cs, gi0 - l_off);
    const size_t YB = (size_t)m.nsp * N * sizeof(real);
    cp(m.mech, h.mech, sizeof(MechData));
    for (int b = 0; b < 2; b++) cp(m.Ys[b], h.Ys[0].data(), YB);
    cp(m.As, h.As.data(), YB);
    cp(m.Bs, h.Bs.data(), YB);
    cp(m.Fs, h.Fs.data(), YB);
    cp(m.betas, h.betas.data(), YB);
    if (m.dSdxs[0])
      for (int b = 0; b < 2; b++) {
        cp(m.dSdxs[b], h.dSdxs[0].data(), YB);
        cp(m.dSdys[b], h.dSdys[0].data(), YB);
      }
  }
  scen_host.cfl = cs.cfg.CFL_Scenario.pack();
  scen_host.beta = cs.cfg.beta_Scenario.pack();
  scen_host.CFL = cs.cfg.CFL;
  scen_host.beta0 = cs.cfg.beta0;
  cp(m.scen, &scen_host, sizeof(ScenarioTables));
  DevScalars s0{};
  const double d0 = dt;
  const double one = 1.0;  // slot 1 accumulates step 0's min; slot 2 is reset by step 0
  unsigned long long b0, b1;
  std::memcpy(&b0, &d0, 8);
  std::memcpy(&b1, &one, 8);
  dt_set_host(s0, 0, b0);
  dt_set_host(s0, 1, b1);
  dt_set_host(s0, 2, b1);
  if (make_params(last_iter + iter).lag_dt) {
    // lagged dt: the first step runs with dt; slot 0's MIN stands for the
    // previous step's (the host's dt_lag, or dt before any step)
    s0.dt_lag[0] = b0;
    const double dl = dt_lag > 0 ? dt_lag : dt;
    unsigned long long bl;
    std::memcpy(&bl, &dl, 8);
    dt_set_host(s0, 0, bl);
  }
  s0.time_part = 0.0;
  s0.iter[0] = s0.iter[1] = s0.iter[2] = (double)(last_iter + iter);
  {
    const StepParams Pi = make_params(last_iter + iter);
    for (int q = 0; q < 3; q++) {
      s0.beta_min[q] = Pi.beta_min;
      s0.cfl_min[q] = Pi.CFL_min;
    }
  }
  time_offset = -cur_time_part;
  last_dev_time = 0.0;
  *m.sc_host = s0;
  cp(m.sc, m.sc_host, sizeof(DevScalars));
  m.sc_mirrored = false;
  HIP_CHECK(hipStreamSynchronize(st));
  nstep = 0;
  abuf = 0;
  sbuf = 0;
  dsbuf = 0;
  pbuf = 0;
}

void DeviceSolver::set_lean_plain(bool on) {
  lean_plain = on;
  if (!lean_ok) return;
  std::vector<uint8_t> b = lean_flags(h, cs.cfg.ProblemType);
  if (!on)
    for (auto& x : b) x &= (uint8_t)~LB_PLAIN;
  lean_bytes = b;
  HIP_CHECK(hipMemcpyAsync(impl->lb, lean_bytes.data(), lean_bytes.size(), hipMemcpyHostToDevice, impl->stream));
  HIP_CHECK(hipStreamSynchronize(impl->stream));
}

void DeviceSolver::lean_materialize() {
  p2p_complete();
  Impl& m = *impl;
  StepParams P = make_params(last_iter + iter);
  P.nx = h.nx;
  P.ny = h.ny;
  LeanSoA L = m.lean_view(h, sbuf, abuf, dsbuf, pbuf, false);
  SoA g = m.view(h, sbuf, abuf, dsbuf, pbuf);
  const unsigned nb = (unsigned)((h.N + BLOCK - 1) / BLOCK);
  hipLaunchKernelGGL(hf2d_lean_materialize, dim3(nb), dim3(BLOCK), 0, m.stream, P, L, g, 0L, h.N);
  HIP_CHECK(hipGetLastError());
  lean_state = 0;
}

// Lean N-S -> generic record: the split fill F_m over every cell from the
// lean state (Sp^m, level m-1 primitives), i.e. exactly the fill the split
// stepper ran (committed S, A/B/F, SrcAdd, level-m primitives, Diff and
// gradients); its dt is already in the next slot (no dt update here).
void DeviceSolver::lns_materialize() {
  p2p_complete();
  Impl& m = *impl;
  StepParams P = make_params(last_iter + iter);
  P.nx = h.nx;
  P.ny = h.ny;
  P.i0 = l_off;
  P.i1 = l_off + (gi1 - gi0);
  P.gx0 = gi0 - l_off;
  P.species = m.species;
  P.scen = m.scen;
  if (m.mech) {
    // lean mechanism path: the split (lazy) fill F_{m+1} from Sp^{m+1}, its
    // post-kinetics species and the level-m primitives / transport; the
    // lagged k of its skip test is the state of level m
    SoA sin = m.view(h, 1 - sbuf, abuf, dsbuf, 1 - pbuf);
    m.mech_view(sin, sbuf, dsbuf);
    real* const mux[2] = {m.mu, m.mu2};
    real* const lamx[2] = {m.lam, m.lam2};
    real* const mutx[2] = {m.mu_t, m.mu_t2};
    real* const cpx[2] = {m.CP, m.CP2};
    real* const kkx[2] = {m.kk, m.kk2};
    real* const px[2] = {m.p, m.p2};
    sin.mu = mux[1 - cbuf];
    sin.lam = lamx[1 - cbuf];
    sin.mu_t = mutx[1 - cbuf];
    sin.CP = cpx[cbuf];
    sin.kk = kkx[cbuf];
    sin.p = px[cbuf];
    SoA out = m.view(h, sbuf, abuf, dsbuf, pbuf);
    const long c0 = (long)P.i0 * P.ny, c1 = (long)P.i1 * P.ny;
    const unsigned nb = (unsigned)((c1 - c0 + BLOCK - 1) / BLOCK);
    // (the split fill F_{m+1} belongs to step m: its dt is slot m % 3, which
    // step m+1 has not reset yet; SST's point-implicit destruction reads it)
    hipLaunchKernelGGL((hf2d_fill_occ<SK_MECH, 9, 2, true>), dim3(nb), dim3(BLOCK), 0, m.stream, P, sin, sin, out, c0,
                       c1, m.sc, (int)((nstep + 2) % 3), -1, 0, 1);
    HIP_CHECK(hipGetLastError());
    lns_state = 0;
    cbuf = 0;
    return;
  }
  SoA sin = m.view(h, 1 - sbuf, abuf, dsbuf, 1 - pbuf);
  real* const cpx[2] = {m.CP, m.CP2};
  real* const mux[2] = {m.mu, m.mu2};
  real* const lamx[2] = {m.lam, m.lam2};
  real* const kkx[2] = {m.kk, m.kk2};
  real* const mutx[2] = {m.mu_t, m.mu_t2};
  sin.CP = cpx[1 - cbuf];
  sin.mu = mux[1 - cbuf];
  sin.lam = lamx[1 - cbuf];
  sin.kk = kkx[1 - cbuf];
  sin.mu_t = mutx[1 - cbuf];
  SoA out = m.view(h, sbuf, abuf, dsbuf, pbuf);
  const long c0 = (long)P.i0 * P.ny, c1 = (long)P.i1 * P.ny;
  const unsigned nb = (unsigned)((c1 - c0 + BLOCK - 1) / BLOCK);
  // (the split fill F_{m+1} belongs to step m: its dt is slot m % 3, which
  // step m+1 has not reset yet; SST's point-implicit destruction reads it)
  if (sk_mode == SK_SGT)
    hipLaunchKernelGGL((hf2d_fill<SK_SGT, 1>), dim3(nb), dim3(BLOCK), 0, m.stream, P, sin, sin, out, c0, c1, m.sc,
                       (int)((nstep + 2) % 3), -1, 0, 1);
  else
    hipLaunchKernelGGL((hf2d_fill<SK_SGL, 1>), dim3(nb), dim3(BLOCK), 0, m.stream, P, sin, sin, out, c0, c1, m.sc,
                       (int)(nstep % 3), -1, 0, 1);
  HIP_CHECK(hipGetLastError());
  lns_state = 0;
  cbuf = 0;
}

void DeviceSolver::download(Field& J) {
  flush_pending();
  p2p_complete();
  HIP_CHECK(hipSetDevice(dev));
  Impl& m = *impl;
  if (lean_state) lean_materialize();
  if (lns_state) lns_materialize();
  hipStream_t st = m.stream;
  const long N = h.N;
  auto cp = [&](void* d, const void* s, size_t bytes) { HIP_CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToHost, st)); };
  const size_t EQB = NEQ * N * sizeof(real), SB = N * sizeof(real);
  cp(h.S[0].data(), m.S[sbuf], EQB);
  cp(h.A.data(), m.A[abuf], EQB);
  cp(h.B.data(), m.B[abuf], EQB);
  cp(h.dSdx[0].data(), m.dSdx[dsbuf], EQB);
  cp(h.dSdy[0].data(), m.dSdy[dsbuf], EQB);
  cp(h.U[0].data(), m.U[pbuf], SB);
  cp(h.V[0].data(), m.V[pbuf], SB);
  cp(h.Tg[0].data(), m.Tg[pbuf], SB);
  cp(h.F.data(), m.F, EQB);
  cp(h.Src.data(), m.Src, EQB);
  cp(h.SrcAdd.data(), m.SrcAdd, EQB);
  cp(h.beta.data(), m.beta, EQB);
  cp(h.p.data(), m.p, SB);
  cp(h.kk.data(), m.kk, SB);
  cp(h.R.data(), m.R, SB);
  cp(h.CP.data(), m.CP, SB);
  cp(h.lam.data(), m.lam, SB);
  cp(h.mu.data(), m.mu, SB);
  cp(h.mu_t.data(), m.mu_t, SB);
  cp(h.lam_t.data(), m.lam_t, SB);
  cp(h.Diff.data(), m.Diff, SB);
  cp(h.Y.data(), m.Y, NSPEC * SB);
  cp(h.y_plus.data(), m.y_plus, SB);
  cp(h.Re_local.data(), m.Re_local, SB);
  cp(h.Q_conv.data(), m.Q_conv, SB);
  cp(h.grad.data(), m.grad, NGRAD * SB);
  cp(h.CT.data(), m.CT, N * sizeof(u64));
  if (h.mech) cp(h.Ys[0].data(), m.Ys[sbuf], (size_t)m.nsp * N * sizeof(real));
  HIP_CHECK(hipStreamSynchronize(st));
  h.to_field(J, gi0 - l_off, l_off, l_off + (gi1 - gi0), 0, 0);
  h.mech_to_case(cs, gi0 - l_off, l_off, l_off + (gi1 - gi0), 0);
}

void DeviceSolver::on_cycle_roll() { time_offset = last_dev_time; }

void DeviceSolver::sample_monitors(std::vector<MonitorPoint>& mp) {
  if (mp.empty()) return;
  flush_pending();
  p2p_complete();
  Impl& m = *impl;
  if (lns_state) lns_materialize();
  const int n = (int)mp.size();
  std::vector<long> idx(n, -1);
  for (int q = 0; q < n; q++) {
    const int i = (int)(mp[q].x / cs.cfg.dx), j = (int)(mp[q].y / cs.cfg.dy);
    if (cs.J.in(i, j) && i >= gi0 && i < gi1) idx[q] = (long)(i - gi0 + l_off) * h.ny + j;
  }
  if ((int)probe_idx_host.size() != n) {
    probe_idx_host.assign(n, -2);
    probe_buf_host.assign(2 * n, 0.0);
    impl->probe_idx = m.mem.alloc<long>(n);
    impl->probe_out = m.mem.alloc<real>(2 * n);
    HIP_CHECK(hipDeviceSynchronize());
  }
  if (idx != probe_idx_host) {
    probe_idx_host = idx;
    HIP_CHECK(hipMemcpyAsync(m.probe_idx, probe_idx_host.data(), n * sizeof(long), hipMemcpyHostToDevice, m.stream));
  }
  // current pressure: the lean arrays while they are authoritative
  const real* p = lean_state ? m.P2[pbuf] : m.p;
  hipLaunchKernelGGL(hf2d_probe_gather, dim3((n + 63) / 64), dim3(64), 0, m.stream, m.probe_idx, n, p, m.Tg[pbuf],
                     m.probe_out);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(probe_buf_host.data(), m.probe_out, 2 * n * sizeof(real), hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  for (int q = 0; q < n; q++) {
    real pv = probe_buf_host[2 * q], Tv = probe_buf_host[2 * q + 1];
    const int i = (int)(mp[q].x / cs.cfg.dx), j = (int)(mp[q].y / cs.cfg.dy);
    if (comm->size() > 1) {   // exactly one rank owns the probe
      pv = comm->allreduce_sum(pv);
      Tv = comm->allreduce_sum(Tv);
    } else if (!cs.J.in(i, j)) {
      continue;
    }
    mp[q].p = pv;
    mp[q].T = Tv;
  }
}

void DeviceSolver::poison_cell(int gi, int j) {
  flush_pending();
  Impl& m = *impl;
  if (lns_state) lns_materialize();
  const long idx = (long)(gi - gi0 + l_off) * h.ny + j;
  static const real bad = -1.0e30;
  HIP_CHECK(hipMemcpyAsync(m.S[sbuf] + (long)I_RHOE * h.N + idx, &bad, sizeof bad, hipMemcpyHostToDevice, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
}

// driver phases as roctx ranges (rocprofv3 --marker-trace)
void DeviceSolver::trace_push(const char* name) { roctxRangePush(name); }
void DeviceSolver::trace_pop() { roctxRangePop(); }

void DeviceSolver::sync_scalars() {
  flush_pending();
  p2p_complete();
  Impl& m = *impl;
  if (m.sc_mirrored) {
    // the last step wrote the mirror (host_tail).  It refreshes ONLY the dt
    // shards, dt_bits, dt_lag, time_part and neg_T of sc_host; the other
    // DevScalars fields there (iter, scenario beta / CFL, dt_val, hot counts)
    // are stale, so this function must read nothing else below this point
    // (hf2d_scalars_out / the memcpy refresh the whole header).
  } else if (m.sc_kernel) {
    hipLaunchKernelGGL(hf2d_scalars_out, dim3(1), dim3(WAVE), 0, m.stream, m.sc, m.sc_host, (int)(nstep % 3));
    HIP_CHECK(hipGetLastError());
  } else {
    HIP_CHECK(hipMemcpyAsync(m.sc_host, m.sc, sizeof(DevScalars), hipMemcpyDeviceToHost, m.stream));
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));
  const int slot = nstep % 3;
  const unsigned long long db = dt_get_host(*m.sc_host, slot);
  if (make_params(last_iter + iter).lag_dt) {   // next step's dt, and the MIN it hands on
    std::memcpy(&dt, &m.sc_host->dt_lag[slot], 8);
    std::memcpy(&dt_lag, &db, 8);
  } else {
    std::memcpy(&dt, &db, 8);
  }
  cur_time_part = m.sc_host->time_part - time_offset;
  last_dev_time = m.sc_host->time_part;
  const int err = comm->allreduce_max_int(m.sc_host->neg_T);
  if (err & 2) {
    char b[256];
    std::snprintf(b, sizeof b, "ERROR: P2P halo exchange timed out (peer rank not responding) before iteration %ld",
                  last_iter + iter);
    throw std::runtime_error(b);
  }
  if (err & LNS_SKIP_ERR) {
    char b[256];
    std::snprintf(b, sizeof b, "ERROR: lean N-S step: FillNode2D skipped a node (rho = 0 or k < 1) before iteration %ld",
                  last_iter + iter);
    throw std::runtime_error(b);
  }
  if (err) {
    char b[256];
    std::snprintf(b, sizeof b, "ERROR: Computational unstability (Tg < 0) before iteration %ld", last_iter + iter);
    throw std::runtime_error(b);
  }
}

// Called at each outer-cycle boundary by the driver (time_part restarts).
void DeviceSolver::cycle_update() {
  flush_pending();
  p2p_complete();
  Impl& m = *impl;
  if (lns_state) lns_materialize();
  if (cs.cfg.ProblemType == SM_NS && cs.cfg.semantics != Semantics::SERIAL) {
    SoA s = m.view(h, sbuf, abuf, dsbuf, pbuf);
    const int nw = (int)h.wall_own.size(), nall = (int)cs.wall_nodes.size();
    std::vector<real> v(nw);
    std::vector<uint8_t> g(nw);
    if (nw) {
      hipLaunchKernelGGL(hf2d_wall_uw, dim3((nw + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, m.stream, s, m.wall_own, nw,
                         m.wall_uw, m.wall_ok);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(v.data(), m.wall_uw, nw * sizeof(real), hipMemcpyDeviceToHost, m.stream));
      HIP_CHECK(hipMemcpyAsync(g.data(), m.wall_ok, nw, hipMemcpyDeviceToHost, m.stream));
      HIP_CHECK(hipStreamSynchronize(m.stream));
    }
    std::vector<int32_t> sl;
    std::vector<real> vals;
    for (int k = 0; k < nw; k++)
      if (g[k]) {
        sl.push_back(h.wall_own_slot[k]);
        vals.push_back(v[k]);
      }
    std::vector<real> uw;
    std::vector<uint8_t> ok;
    merge_wall_uw(sl, vals, uw, ok);
    if (nall) {
      HIP_CHECK(hipMemcpyAsync(m.uw_all, uw.data(), nall * sizeof(real), hipMemcpyHostToDevice, m.stream));
      HIP_CHECK(hipMemcpyAsync(m.uw_all_ok, ok.data(), nall, hipMemcpyHostToDevice, m.stream));
      const long c0 = (long)l_off * h.ny, c1 = (long)(l_off + (gi1 - gi0)) * h.ny;
      const unsigned nb = (unsigned)((c1 - c0 + BLOCK - 1) / BLOCK);
      hipLaunchKernelGGL(hf2d_yplus, dim3(nb), dim3(BLOCK), 0, m.stream, s, c0, c1, m.uw_all, m.uw_all_ok);
      HIP_CHECK(hipGetLastError());
    }
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));
}

// Host-side reductions of the driver over RCCL (output steps only).
struct RcclHostComm : Comm {
  ncclComm_t c;
  hipStream_t st;
  int r, n;
  double* buf = nullptr;
  RcclHostComm(ncclComm_t c_, hipStream_t s_, int r_, int n_) : c(c_), st(s_), r(r_), n(n_) {
    HIP_CHECK(hipMalloc((void**)&buf, sizeof(ResidualPack) * (n + 1) + 64));
  }
  ~RcclHostComm() override { (void)hipFree(buf); }
  int rank() const override { return r; }
  int size() const override { return n; }
  double reduce1(double v, ncclRedOp_t op) {
    HIP_CHECK(hipMemcpyAsync(buf, &v, 8, hipMemcpyHostToDevice, st));
    NCCL_CHECK(ncclAllReduce(buf, buf, 1, ncclDouble, op, c, st));
    HIP_CHECK(hipMemcpyAsync(&v, buf, 8, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return v;
  }
  real allreduce_min(real v) override { return reduce1(v, ncclMin); }
  real allreduce_sum(real v) override { return reduce1(v, ncclSum); }
  int allreduce_max_int(int v) override { return (int)reduce1((double)v, ncclMax); }
  // variable-size all-gather through a device staging buffer: the sizes
  // first, then every rank's bytes padded to the largest (outputs only:
  // row lengths, ghost columns and integral terms once per outer cycle)
  std::vector<std::string> allgather_bytes(const std::string& mine) override {
    long long* dsz = (long long*)buf;
    const long long me = (long long)mine.size();
    HIP_CHECK(hipMemcpyAsync(dsz, &me, sizeof me, hipMemcpyHostToDevice, st));
    NCCL_CHECK(ncclAllGather(dsz, dsz + 1, 1, ncclInt64, c, st));
    std::vector<long long> sz(n);
    HIP_CHECK(hipMemcpyAsync(sz.data(), dsz + 1, sizeof(long long) * n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    size_t maxb = 1;
    for (long long v : sz) maxb = std::max(maxb, (size_t)v);
    char* stage = nullptr;
    HIP_CHECK(hipMalloc((void**)&stage, maxb * (n + 1)));
    if (me) HIP_CHECK(hipMemcpyAsync(stage, mine.data(), (size_t)me, hipMemcpyHostToDevice, st));
    NCCL_CHECK(ncclAllGather(stage, stage + maxb, maxb, ncclChar, c, st));
    std::string flat(maxb * n, '\0');
    HIP_CHECK(hipMemcpyAsync(&flat[0], stage + maxb, maxb * n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipFree(stage));
    std::vector<std::string> all(n);
    for (int q = 0; q < n; q++) all[q] = flat.substr((size_t)q * maxb, (size_t)sz[q]);
    return all;
  }
  void allreduce_residual(ResidualPack& p) override {
    std::vector<ResidualPack> all(n);
    char* dbuf = (char*)buf;
    HIP_CHECK(hipMemcpyAsync(dbuf, &p, sizeof(ResidualPack), hipMemcpyHostToDevice, st));
    NCCL_CHECK(ncclAllGather(dbuf, dbuf + sizeof(ResidualPack), sizeof(ResidualPack), ncclChar, c, st));
    HIP_CHECK(hipMemcpyAsync(all.data(), dbuf + sizeof(ResidualPack), sizeof(ResidualPack) * n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    ResidualPack a = all[0];
    for (int q = 1; q < n; q++) residual_merge_lex(a, all[q]);
    p = a;
  }
};

std::string DeviceSolver::nccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

void DeviceSolver::init_comm(const std::string& uid, int rank, int nranks) {
  HIP_CHECK(hipSetDevice(dev));
  ncclUniqueId id;
  if (uid.size() != sizeof(id.internal)) throw std::runtime_error("bad RCCL unique id size");
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  NCCL_CHECK(ncclCommInitRank(&impl->comm, nranks, id, rank));
  impl->rank = rank;
  impl->nranks = nranks;
  impl->dt_recv = impl->mem.alloc<double>(nranks);
  HIP_CHECK(hipDeviceSynchronize());
  host_comm.reset(new RcclHostComm(impl->comm, impl->stream, rank, nranks));
  comm = host_comm.get();
}

void DeviceSolver::init_local(std::shared_ptr<LocalGroup> g, int rank) {
  impl->local = g;
  impl->rank = rank;
  impl->nranks = g->n;
  impl->dt_recv = impl->mem.alloc<double>(g->n);
  HIP_CHECK(hipDeviceSynchronize());
  host_comm.reset(new LocalHostComm(g, rank));
  comm = host_comm.get();
}

namespace {
struct P2PDesc {
  uint32_t magic;
  int32_t pid, device, rank, nranks, pad;
  uint64_t ptr, bytes;
  char handle[HIP_IPC_HANDLE_SIZE];
};
constexpr uint32_t P2P_MAGIC = 0x68663270;   // "hf2p"
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

std::string DeviceSolver::p2p_export(int rank, int nranks) {
  HIP_CHECK(hipSetDevice(dev));
  Impl& m = *impl;
  if (m.p2p.base) throw std::runtime_error("p2p_export: mailbox already exported");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("p2p_export: bad rank/nranks");
  m.rank = rank;
  m.nranks = nranks;
  Impl::P2P& p = m.p2p;
  p.off_dtr = align_up((size_t)nranks * 8, 256);
  p.off_recv = align_up(p.off_dtr + (size_t)2 * nranks * 8, 256);
  p.bytes = p.off_recv + (size_t)4 * m.halo_cap * sizeof(real);
  void* b = nullptr;
  HIP_CHECK(hipExtMallocWithFlags(&b, p.bytes, hipDeviceMallocFinegrained));
  m.mem.ptrs.push_back(b);
  p.base = (char*)b;
  HIP_CHECK(hipMemset(p.base, 0, p.bytes));
  p.seq = m.mem.alloc<unsigned long long>(1);
  p.done = m.mem.alloc<unsigned>(FX_DONE_WORDS);
  HIP_CHECK(hipDeviceSynchronize());
  P2PDesc d{};
  d.magic = P2P_MAGIC;
  d.pid = (int32_t)getpid();
  d.device = dev;
  d.rank = rank;
  d.nranks = nranks;
  d.ptr = (uint64_t)(uintptr_t)p.base;
  d.bytes = p.bytes;
  hipIpcMemHandle_t h;
  HIP_CHECK(hipIpcGetMemHandle(&h, p.base));
  std::memcpy(d.handle, &h, sizeof(h));
  return std::string((const char*)&d, sizeof d);
}

// One-GPU stand-in for the multi-GPU mailbox exchange (timing only,
// tools/exchange_loopback.py): this strip plays rank `rank` of `nranks`,
// every peer has already published its step (flags at the maximum, dt 1.0),
// and the neighbours' mailboxes are this rank's own (Impl::P2P::push_base:
// the left edge push lands in the left-ghost mailbox, zero-gradient ghosts).
// A step then does every store, publication, poll and ghost staging of a
// real exchange, without a second strip on the GPU and without waiting --
// what remains is the exchange's own cost on this device (the xGMI link
// latency is not in it).
void DeviceSolver::p2p_loopback(int rank, int nranks) {
  if (nranks < 2 || rank < 0 || rank >= nranks) throw std::runtime_error("p2p_loopback: bad rank/nranks");
  (void)p2p_export(rank, nranks);
  HIP_CHECK(hipSetDevice(dev));
  Impl& m = *impl;
  Impl::P2P& p = m.p2p;
  p.peer_base.assign(nranks, p.base);
  std::vector<unsigned long long> flags(nranks, ~0ull);
  flags[rank] = 0;
  std::vector<double> dtr(2 * (size_t)nranks, 1.0);
  HIP_CHECK(hipMemcpy(p.base, flags.data(), nranks * sizeof(unsigned long long), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(p.base + p.off_dtr, dtr.data(), dtr.size() * sizeof(double), hipMemcpyHostToDevice));
  std::vector<unsigned long long*> fl(nranks, (unsigned long long*)p.base);
  std::vector<double*> dr(nranks, (double*)(p.base + p.off_dtr));
  p.d_flags = m.mem.alloc<unsigned long long*>(nranks);
  p.d_dtr = m.mem.alloc<double*>(nranks);
  if (!m.lc_dev) m.lc_dev = m.mem.alloc<ColList>(2);
  HIP_CHECK(hipMemcpy(p.d_flags, fl.data(), nranks * sizeof(void*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(p.d_dtr, dr.data(), nranks * sizeof(void*), hipMemcpyHostToDevice));
  p.loop = true;
  p.on = true;
}

void DeviceSolver::p2p_import(const std::vector<std::string>& descs) {
  HIP_CHECK(hipSetDevice(dev));
  Impl& m = *impl;
  Impl::P2P& p = m.p2p;
  if (!p.base) throw std::runtime_error("p2p_import before p2p_export");
  if ((int)descs.size() != m.nranks) throw std::runtime_error("p2p_import: need one descriptor per rank");
  if (p2p_queue_check) {
    // In-process ranks on one device (virtual ranks: tests, one-GPU boxes).
    // Every rank's exchange kernel ends in a workgroup that spins until all
    // peers have published, so the ranks' kernels must run concurrently.  HIP
    // maps a process's streams onto at most GPU_MAX_HW_QUEUES hardware queues
    // per device (default 4) and past that puts two streams on one queue,
    // whose packets run in order: a spinning kernel then holds back the peer
    // kernel queued behind it until the bounded wait expires ("rank 0 timed
    // out waiting for its peers", the round-5 4-rank probe).  Measured on
    // MI355X (tools/hwq_probe.py, profiles/hwq_probe_r06.md): n ranks in one
    // process co-schedule iff GPU_MAX_HW_QUEUES >= n + 1 (3 and 4 queues,
    // 4 and 8, 8 and 16 pass; 4 and 4, 8 and 8 time out).  Separate
    // processes (the multi-GPU layout) have queues of their own.
    int local = 0;
    for (const std::string& s : descs) {
      P2PDesc d;
      if (s.size() != sizeof d) continue;
      std::memcpy(&d, s.data(), sizeof d);
      local += (d.pid == (int32_t)getpid() && d.device == dev) ? 1 : 0;
    }
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    const int hwq = (q && std::atoi(q) > 0) ? std::atoi(q) : 4;
    if (local > 1 && local + 1 > hwq)
      throw std::runtime_error("p2p_import: " + std::to_string(local) + " mailbox ranks share device " +
                               std::to_string(dev) + " in one process, which has " + std::to_string(hwq) +
                               " HIP hardware queues (GPU_MAX_HW_QUEUES); their exchange kernels wait for each "
                               "other, so each rank needs a queue of its own plus one for the default stream: set "
                               "GPU_MAX_HW_QUEUES >= " + std::to_string(local + 1) +
                               " before the first HIP call, or run the ranks as separate processes");
  }
  p.peer_base.assign(m.nranks, nullptr);
  for (int q = 0; q < m.nranks; q++) {
    P2PDesc d;
    if (descs[q].size() != sizeof d) throw std::runtime_error("p2p_import: bad descriptor size");
    std::memcpy(&d, descs[q].data(), sizeof d);
    if (d.magic != P2P_MAGIC || d.rank != q || d.nranks != m.nranks || d.bytes != p.bytes)
      throw std::runtime_error("p2p_import: descriptor mismatch (rank " + std::to_string(q) + ")");
    if (q == m.rank) {
      p.peer_base[q] = p.base;
    } else if (d.pid == (int32_t)getpid()) {   // in-process virtual rank
      if (d.device != dev) {
        const hipError_t e = hipDeviceEnablePeerAccess(d.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
        (void)hipGetLastError();
      }
      p.peer_base[q] = (char*)(uintptr_t)d.ptr;
    } else {
      hipIpcMemHandle_t h;
      std::memcpy(&h, d.handle, sizeof h);
      void* ptr = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
      p.opened.push_back(ptr);
      p.peer_base[q] = (char*)ptr;
    }
  }
  std::vector<unsigned long long*> fl(m.nranks);
  std::vector<double*> dr(m.nranks);
  for (int q = 0; q < m.nranks; q++) {
    fl[q] = (unsigned long long*)p.peer_base[q];
    dr[q] = (double*)(p.peer_base[q] + p.off_dtr);
  }
  p.d_flags = m.mem.alloc<unsigned long long*>(m.nranks);
  p.d_dtr = m.mem.alloc<double*>(m.nranks);
  if (!m.lc_dev) m.lc_dev = m.mem.alloc<ColList>(2);   // (fused lean N-S ghost prologue lists)
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(p.d_flags, fl.data(), m.nranks * sizeof(void*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(p.d_dtr, dr.data(), m.nranks * sizeof(void*), hipMemcpyHostToDevice));
  p.on = m.nranks > 1;
}

bool DeviceSolver::p2p_active() const { return impl->p2p.on; }

void DeviceSolver::p2p_set(bool on) {
  flush_pending();
  p2p_complete();
  lns_last_valid = false;
  if (on && (impl->p2p.peer_base.empty() || impl->nranks < 2)) throw std::runtime_error("p2p_set: no imported peers");
  impl->p2p.on = on;
  graph.reset();   // captured exchanges belong to the old transport
}

int DeviceSolver::comm_rank() const { return impl->rank; }
int DeviceSolver::comm_size() const { return impl->nranks; }

// Halo exchange of one field group with RCCL send/recv to the strip
// neighbours (rank-1 owns the columns to the left).  dt_slot >= 0: the
// same RCCL group also sends this rank's dt of that slot to every other rank
// and unpack folds the MIN in -- one grouped p2p launch per step instead of a
// send/recv group plus an all-reduce.
// device columns of the fields a halo group carries (pack order)
int DeviceSolver::split_mode() const {
  return impl->mech ? SK_MECH : (cs.cfg.ProblemType == SM_NS && sgl) ? sk_mode : SK_GENERIC;
}

void DeviceSolver::halo_fields(int group, std::vector<real*>& f, bool full) const {
  std::vector<unsigned char> o;
  halo_fields(group, f, o, full);
}

void DeviceSolver::halo_fields(int group, std::vector<real*>& f, std::vector<unsigned char>& o, bool full) const {
  const Impl& m = *impl;
  const long N = h.N;
  f.clear();
  o.clear();
  if (group == CpuSolver::HALO_LNS) {
    // lean N-S / mechanism strips (two ghost columns): what the next lean step
    // reads of them -- the inner ghost column is a ring cell (its fill reads
    // its predicted state, lagged primitives, transport and thermodynamic
    // state), the outer one only the neighbour values of that fill (state,
    // species, lagged U, V, T)
    const int cb = cbuf;
    auto two = [&](real* p) {
      f.push_back(p);
      o.push_back(0);
      f.push_back(p);
      o.push_back(1);
    };
    auto one = [&](real* p) {
      f.push_back(p);
      o.push_back(0);
    };
    for (int k = 0; k < NEQ; k++)
      if (sk_live(m.mech ? SK_MECH : sk_mode, k)) two(m.S[1 - sbuf] + (long)k * N);
    two(m.U[1 - pbuf]);
    two(m.V[1 - pbuf]);
    two(m.Tg[1 - pbuf]);
    real* const mux[2] = {m.mu, m.mu2};
    real* const lamx[2] = {m.lam, m.lam2};
    real* const mutx[2] = {m.mu_t, m.mu_t2};
    real* const cpx[2] = {m.CP, m.CP2};
    real* const kkx[2] = {m.kk, m.kk2};
    one(mux[1 - cb]);
    one(lamx[1 - cb]);
    one(mutx[1 - cb]);
    one(cpx[1 - cb]);
    one(kkx[1 - cb]);
    if (m.mech) {
      real* const px[2] = {m.p, m.p2};
      one(px[1 - cb]);
      one(m.Tst[1 - cb]);
      for (int q = 0; q < m.nsp; q++) two(m.Ys[sbuf] + (long)q * N);
    }
    if (any_cauchy_x) {   // dS/dx of the ghost column (Cauchy neighbours of the edge cells)
      for (int k = 0; k < NEQ; k++)
        if (sk_live(m.mech ? SK_MECH : sk_mode, k)) one(m.dSdx[dsbuf] + (long)k * N);
      if (m.dSdxs[0])
        for (int q = 0; q < m.nsp; q++) one(m.dSdxs[dsbuf] + (long)q * N);
    }
    return;
  }
  full = full || !halo_compact;
  const int mode = split_mode();
  auto add_eq = [&](real* base) {
    for (int k = 0; k < NEQ; k++) f.push_back(base + (long)k * N);
  };
  if (group == CpuSolver::HALO_LEAN) {
    // single gas: the species (and their pre-chemistry copies) are +0 on
    // every rank; dS/dx only travels if some node applies d2/dx2 = 0
    const bool sg = lean_sg && lean_sg_ok;
    for (int k = 0; k < (sg ? 4 : 4 + NCOMP); k++) f.push_back(m.S[sbuf] + (long)k * N);
    if (!sg)
      for (int k = 0; k < NCOMP; k++) f.push_back(m.Spre[pbuf] + (long)k * N);
    f.push_back(m.U[pbuf]);
    f.push_back(m.V[pbuf]);
    f.push_back(m.P2[pbuf]);
    if (lean_has_cauchy_x) add_eq(m.dSdx[dsbuf]);
  } else if (group == CpuSolver::HALO_MID) {
    // the predicted state as the N-S fill reads it of an x neighbour
    // (stepkern.hpp fill_compute: Sn of rho, the species slots, k and eps);
    // mechanism strips also react their ghost columns, which reads rho, rhoU,
    // rhoV and rhoE (chem_fast_dev.hpp chem_cell)
    for (int k = 0; k < NEQ; k++)
      if (full || k == 0 || (mode == SK_MECH && k < 4) || (k >= 4 && sk_live(mode, k)))
        f.push_back(m.S[1 - sbuf] + (long)k * N);
    for (int q = 0; q < m.nsp; q++) f.push_back(m.Ys[1 - sbuf] + (long)q * N);
  } else if (group == CpuSolver::HALO_QDIR) {
    for (int d = 0; d < 4; d++) f.push_back(m.qdir + (long)d * N);
  } else {
    // what the next split step reads of a ghost column: the predictor's S
    // and x flux A of the live equations (stepkern.hpp predict_core: SL/SR,
    // AL/AR; the y flux B only along the own column), dS/dx only where a node
    // applies d2/dx2 = 0, the fill's previous U/V/T and the wall heat flux's
    // conductivities; the mechanism species block likewise
    for (int k = 0; k < NEQ; k++)
      if (full || sk_live(mode, k)) f.push_back(m.S[sbuf] + (long)k * N);
    for (int k = 0; k < NEQ; k++)
      if (full || sk_live(mode, k)) f.push_back(m.A[abuf] + (long)k * N);
    if (full) add_eq(m.B[abuf]);
    if (full || any_cauchy_x)
      for (int k = 0; k < NEQ; k++)
        if (full || sk_live(mode, k)) f.push_back(m.dSdx[dsbuf] + (long)k * N);
    f.push_back(m.U[pbuf]);
    f.push_back(m.V[pbuf]);
    f.push_back(m.Tg[pbuf]);
    f.push_back(m.lam);
    f.push_back(m.lam_t);
    for (int q = 0; q < m.nsp; q++) {
      f.push_back(m.Ys[sbuf] + (long)q * N);
      f.push_back(m.As + (long)q * N);
      if (full) f.push_back(m.Bs + (long)q * N);
      if (m.dSdxs[0] && (full || any_cauchy_x)) f.push_back(m.dSdxs[dsbuf] + (long)q * N);
    }
  }
}

void DeviceSolver::exchange(int group, int dt_slot, void* on_stream, bool full) {
  Impl& m = *impl;
  p2p_complete();
  lns_last_valid = false;
  if ((!m.comm && !m.local && !m.p2p.on) || m.nranks == 1) return;
  const int ny = h.ny;
  std::vector<real*> fl;
  std::vector<unsigned char> fo;
  halo_fields(group, fl, fo, full);
  if (group == CpuSolver::HALO_STATE) ghost_mode = (full || !halo_compact) ? -1 : split_mode();
  if (group == CpuSolver::HALO_LNS) ghost_stale = true;   // lean representation in the ghosts
  else if (group == CpuSolver::HALO_STATE) ghost_stale = false;
  if (fl.size() > (size_t)MAX_HALO_FIELDS) throw std::runtime_error("halo: too many exchanged fields");
  ColList L;
  L.nf = (int)fl.size();
  for (int k = 0; k < L.nf; k++) {
    L.f[k] = fl[k];
    L.o[k] = k < (int)fo.size() ? fo[k] : 0;
  }
  const int cnt = L.nf * ny;
  const unsigned nb2 = (unsigned)((2 * cnt + BLOCK - 1) / BLOCK);
  const int first = l_off, last = l_off + (gi1 - gi0) - 1;
  const bool has_left = gi0 > 0, has_right = gi1 < cs.J.nx;
  const int sides = (has_left ? 1 : 0) | (has_right ? 2 : 0);
  hipStream_t st = on_stream ? (hipStream_t)on_stream : m.stream;
  if (m.p2p.on && p2p_fuse) {
    // multi-workgroup push (the last workgroup publishes, waits and folds the
    // dt), then the multi-workgroup unpack: no single-workgroup copy of the
    // 23-43-field N-S / mechanism halos on the step's critical path
    if (L.nf * ny > m.halo_cap) throw std::runtime_error("p2p halo exceeds mailbox capacity");
    const FusedX X = fused_args();
    hipLaunchKernelGGL(push_kernel(push_per), dim3(push_grid(push_per, cnt)), dim3(BLOCK), 0, st, L, first, last, ny,
                       cnt, X, m.sc,
                       dt_slot >= 0 ? dt_slot : 0, dt_slot >= 0 ? 1 : 0, 1);
    HIP_CHECK(hipGetLastError());
    p2p_mwg_exchanges++;
    if (group == CpuSolver::HALO_LNS && dt_slot >= 0 && lns_ghost_prologue && !on_stream) {
      // the mechanism step's halo: the next mechanism step's edge tiles
      // unpack it (fx_ghost_prologue), any other consumer p2p_complete
      m.lns_pend = L;
      lns_ghost_pending = lns_last_valid = true;
      return;
    }
    hipLaunchKernelGGL(hf2d_p2p_unpack, dim3((unsigned)std::max(1, std::min((2 * cnt + BLOCK - 1) / BLOCK, 1024))),
                       dim3(BLOCK), 0, st, L, l_off - 1, l_off + (gi1 - gi0), ny, cnt, X);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (m.p2p.on) {
    if (L.nf * ny > m.halo_cap) throw std::runtime_error("p2p halo exceeds mailbox capacity");
    Impl::P2P& p = m.p2p;
    P2PArgs a;
    a.L = L;
    a.first = first;
    a.last = last;
    a.ghostL = l_off - 1;
    a.ghostR = l_off + (gi1 - gi0);
    a.ny = ny;
    a.cnt = cnt;
    a.sides = sides;
    a.cap = m.halo_cap;
    a.peer_recv_l = has_left ? p.push_base(0, m.rank, m.halo_cap) : nullptr;
    a.peer_recv_r = has_right ? p.push_base(1, m.rank, m.halo_cap) : nullptr;
    a.my_recv = (real*)(p.base + p.off_recv);
    a.peer_flags = p.d_flags;
    a.peer_dtr = p.d_dtr;
    a.my_flags = (unsigned long long*)p.base;
    a.my_dtr = (double*)(p.base + p.off_dtr);
    a.seq = p.seq;
    a.sc = m.sc;
    a.dslot = dt_slot >= 0 ? dt_slot : 0;
    a.fold_dt = dt_slot >= 0 ? 1 : 0;
    a.rank = m.rank;
    a.nranks = m.nranks;
    hipLaunchKernelGGL(hf2d_p2p_xchg, dim3(1), dim3(P2P_THREADS), 0, m.stream, a);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const bool gather_dt = dt_slot >= 0;
  hipLaunchKernelGGL(hf2d_pack2, dim3(std::max(nb2, 1u)), dim3(BLOCK), 0, st, L, first, last, ny, m.halo_send[0],
                     m.halo_send[1], sides, m.sc, gather_dt ? dt_slot : -1);
  unsigned long long* my_dt = gather_dt ? &m.sc->dt_bits[dt_slot] : nullptr;
  if (m.local) {
    LocalGroup& g = *m.local;
    HIP_CHECK(hipStreamSynchronize(st));
    g.send_l[m.rank] = m.halo_send[0];
    g.send_r[m.rank] = m.halo_send[1];
    g.dt_src[m.rank] = my_dt;
    g.barrier();
    if (gather_dt)
      for (int q = 0; q < m.nranks; q++)
        if (q != m.rank)
          HIP_CHECK(hipMemcpyAsync(m.dt_recv + q, g.dt_src[q], sizeof(double), hipMemcpyDeviceToDevice, st));
    if (has_left)
      HIP_CHECK(hipMemcpyAsync(m.halo_recv[0], g.send_r[m.rank - 1], (size_t)cnt * sizeof(real),
                               hipMemcpyDeviceToDevice, st));
    if (has_right)
      HIP_CHECK(hipMemcpyAsync(m.halo_recv[1], g.send_l[m.rank + 1], (size_t)cnt * sizeof(real),
                               hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    g.barrier();
  } else {
  NCCL_CHECK(ncclGroupStart());
  if (has_left) {
    NCCL_CHECK(ncclSend(m.halo_send[0], cnt, ncclDouble, m.rank - 1, m.comm, st));
    NCCL_CHECK(ncclRecv(m.halo_recv[0], cnt, ncclDouble, m.rank - 1, m.comm, st));
  }
  if (has_right) {
    NCCL_CHECK(ncclSend(m.halo_send[1], cnt, ncclDouble, m.rank + 1, m.comm, st));
    NCCL_CHECK(ncclRecv(m.halo_recv[1], cnt, ncclDouble, m.rank + 1, m.comm, st));
  }
  if (gather_dt)
    for (int q = 0; q < m.nranks; q++)
      if (q != m.rank) {
        NCCL_CHECK(ncclSend(my_dt, 1, ncclDouble, q, m.comm, st));
        NCCL_CHECK(ncclRecv(m.dt_recv + q, 1, ncclDouble, q, m.comm, st));
      }
  NCCL_CHECK(ncclGroupEnd());
  }
  hipLaunchKernelGGL(hf2d_unpack2, dim3(std::max(nb2, 1u)), dim3(BLOCK), 0, st, L, l_off - 1, l_off + (gi1 - gi0), ny,
                     m.halo_recv[0], m.halo_recv[1], sides, m.sc, gather_dt ? dt_slot : 0, m.dt_recv,
                     gather_dt ? m.nranks : 0, m.rank);
  HIP_CHECK(hipGetLastError());
}

namespace {
struct P2PProbe {
  int32_t rank, sides, err, pad;
  uint64_t sent_l, sent_r, recv_l, recv_r;
  double dt;
};
uint64_t fnv1a(const std::vector<real>& v) {
  uint64_t h = 1469598103934665603ULL;
  const unsigned char* p = (const unsigned char*)v.data();
  for (size_t k = 0; k < v.size() * sizeof(real); k++) h = (h ^ p[k]) * 1099511628211ULL;
  return h;
}
constexpr double PROBE_DT0 = 1.0, PROBE_DT_STEP = 0.25;   // rank r offers 1 + r/4: the MIN is 1
}  // namespace

std::string DeviceSolver::p2p_probe() {
  flush_pending();
  p2p_complete();
  HIP_CHECK(hipSetDevice(dev));
  Impl& m = *impl;
  if (!m.p2p.on) throw std::runtime_error("p2p_probe: p2p transport not active");
  hipStream_t st = m.stream;
  const int ny = h.ny;
  const int first = l_off, last = l_off + (gi1 - gi0) - 1, gl = l_off - 1, gr = l_off + (gi1 - gi0);
  const bool has_left = gi0 > 0, has_right = gi1 < cs.J.nx;
  std::vector<real*> fl;
  halo_fields(CpuSolver::HALO_STATE, fl);
  DevScalars saved;
  HIP_CHECK(hipMemcpyAsync(&saved, m.sc, sizeof saved, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  // poison the ghost columns (all-ones bytes: NaN) so a lost delivery shows
  for (real* f : fl) {
    if (has_left) HIP_CHECK(hipMemsetAsync(f + (long)gl * ny, 0xFF, ny * sizeof(real), st));
    if (has_right) HIP_CHECK(hipMemsetAsync(f + (long)gr * ny, 0xFF, ny * sizeof(real), st));
  }
  const unsigned long long tag = [&] {
    const double d = PROBE_DT0 + PROBE_DT_STEP * m.rank;
    unsigned long long b;
    std::memcpy(&b, &d, sizeof b);
    return b;
  }();
  DevScalars tagged = saved;
  dt_set_host(tagged, 0, tag);
  HIP_CHECK(hipMemcpyAsync(m.sc, &tagged, sizeof tagged, hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
  exchange(CpuSolver::HALO_STATE, 0);
  auto column = [&](int col) {
    std::vector<real> v(fl.size() * (size_t)ny);
    for (size_t k = 0; k < fl.size(); k++)
      HIP_CHECK(hipMemcpyAsync(v.data() + k * ny, fl[k] + (long)col * ny, ny * sizeof(real), hipMemcpyDeviceToHost, st));
    return v;
  };
  std::vector<real> sl, sr, rl, rr;
  if (has_left) {
    sl = column(first);
    rl = column(gl);
  }
  if (has_right) {
    sr = column(last);
    rr = column(gr);
  }
  DevScalars after;
  HIP_CHECK(hipMemcpyAsync(&after, m.sc, sizeof after, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  HIP_CHECK(hipMemcpyAsync(m.sc, &saved, sizeof saved, hipMemcpyHostToDevice, st));   // dt slots, error flag
  HIP_CHECK(hipStreamSynchronize(st));
  P2PProbe b{};
  b.rank = m.rank;
  b.sides = (has_left ? 1 : 0) | (has_right ? 2 : 0);
  b.err = after.neg_T & 2;
  b.sent_l = has_left ? fnv1a(sl) : 0;
  b.sent_r = has_right ? fnv1a(sr) : 0;
  b.recv_l = has_left ? fnv1a(rl) : 0;
  b.recv_r = has_right ? fnv1a(rr) : 0;
  const unsigned long long adt = dt_get_host(after, 0);
  std::memcpy(&b.dt, &adt, sizeof b.dt);
  return std::string((const char*)&b, sizeof b);
}

bool DeviceSolver::p2p_probe_ok(const std::vector<std::string>& blobs, int rank, std::string* why) {
  auto bad = [&](const std::string& w) {
    if (why) *why = w;
    return false;
  };
  std::vector<P2PProbe> p(blobs.size());
  for (size_t q = 0; q < blobs.size(); q++) {
    if (blobs[q].size() != sizeof(P2PProbe)) return bad("probe blob of rank " + std::to_string(q) + " missing");
    std::memcpy(&p[q], blobs[q].data(), sizeof(P2PProbe));
  }
  const int n = (int)p.size();
  (void)rank;
  for (int q = 0; q < n; q++) {   // every rank judges all ranks: the verdict is identical everywhere
    if (p[q].rank != q) return bad("probe rank mismatch");
    if (p[q].err) return bad("rank " + std::to_string(q) + " timed out waiting for its peers");
    if (p[q].dt != PROBE_DT0) return bad("rank " + std::to_string(q) + " folded dt " + std::to_string(p[q].dt));
    if ((p[q].sides & 1) && (q == 0 || p[q].recv_l != p[q - 1].sent_r))
      return bad("left halo of rank " + std::to_string(q) + " differs from what rank " + std::to_string(q - 1) + " sent");
    if ((p[q].sides & 2) && (q == n - 1 || p[q].recv_r != p[q + 1].sent_l))
      return bad("right halo of rank " + std::to_string(q) + " differs from what rank " + std::to_string(q + 1) + " sent");
  }
  return true;
}

// p2p failed validation: RCCL (or the in-process group) carries the halos
// from now on; refill the ghost columns the probe poisoned
void DeviceSolver::p2p_fallback() {
  p2p_set(false);
  exchange(CpuSolver::HALO_STATE, -1);
  HIP_CHECK(hipStreamSynchronize(impl->stream));
}

// The global dt MIN alone (comm-overlap steps exchange the halo before the
// interior tiles have produced their dt): RCCL all-reduce (MIN) on the IEEE
// bits of the positive doubles, or the in-process group's device copies.
void DeviceSolver::exchange_dt(int dt_slot) {
  Impl& m = *impl;
  if (m.nranks <= 1) return;
  unsigned long long* my_dt = &m.sc->dt_bits[dt_slot];
  hipLaunchKernelGGL(hf2d_dt_commit, dim3(1), dim3(64), 0, m.stream, m.sc, dt_slot);
  HIP_CHECK(hipGetLastError());
  if (m.comm) {
    NCCL_CHECK(ncclAllReduce(my_dt, my_dt, 1, ncclUint64, ncclMin, m.comm, m.stream));
    return;
  }
  if (!m.local) throw std::runtime_error("exchange_dt: no transport");
  LocalGroup& g = *m.local;
  HIP_CHECK(hipStreamSynchronize(m.stream));
  g.dt_src[m.rank] = my_dt;
  g.barrier();
  for (int q = 0; q < m.nranks; q++)
    if (q != m.rank)
      HIP_CHECK(hipMemcpyAsync(m.dt_recv + q, g.dt_src[q], sizeof(double), hipMemcpyDeviceToDevice, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  g.barrier();
  hipLaunchKernelGGL(hf2d_fold_dt, dim3(1), dim3(64), 0, m.stream, m.sc, dt_slot, m.dt_recv, m.nranks, m.rank);
  HIP_CHECK(hipGetLastError());
}

// Device copy of the fused-exchange arguments for the tile kernels (uploaded
// when they change: at the first fused step, which is never inside a graph
// capture -- the lean entry step runs eagerly)
const FusedX* DeviceSolver::fx_device(const FusedX& X) {
  Impl& m = *impl;
  if (!m.fx_dev) m.fx_dev = m.mem.alloc<FusedX>(1);
  if (!m.fx_dev_valid || std::memcmp(&m.fx_dev_host, &X, sizeof X) != 0) {
    hipStreamCaptureStatus cs_ = hipStreamCaptureStatusNone;
    HIP_CHECK(hipStreamIsCapturing(m.stream, &cs_));
    if (cs_ != hipStreamCaptureStatusNone) throw std::runtime_error("fused exchange arguments changed inside a graph capture");
    HIP_CHECK(hipStreamSynchronize(m.stream));
    HIP_CHECK(hipMemcpy(m.fx_dev, &X, sizeof X, hipMemcpyHostToDevice));
    m.fx_dev_host = X;
    m.fx_dev_valid = true;
  }
  return m.fx_dev;
}

// Device copy of a HALO_LNS list for a fused step's ghost prologue (the two
// buffer parities' lists are uploaded once, outside graph captures; nullptr
// when a new list shows up inside a capture: that step unpacks separately)
namespace {
bool same_list(const ColList& a, const ColList& b) {   // (the entries only: padding bytes are unspecified)
  if (a.nf != b.nf) return false;
  for (int k = 0; k < a.nf; k++)
    if (a.f[k] != b.f[k] || a.o[k] != b.o[k]) return false;
  return true;
}
}  // namespace

const ColList* DeviceSolver::lc_device(const ColList& L) {
  Impl& m = *impl;
  if (!m.lc_dev) return nullptr;   // (allocated by p2p_import)
  for (int k = 0; k < 2; k++)
    if (m.lc_valid[k] && same_list(m.lc_host[k], L)) return m.lc_dev + k;
  // a slot is written once (a captured window may reference it); the two
  // buffer parities' lists fill both, anything else unpacks separately
  if (m.lc_next >= 2) return nullptr;
  hipStreamCaptureStatus cs_ = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(m.stream, &cs_));
  if (cs_ != hipStreamCaptureStatusNone) return nullptr;
  const int k = m.lc_next++;
  m.lc_host[k] = L;
  // stream-ordered from the persistent host copy: no host wait in the step
  HIP_CHECK(hipMemcpyAsync(m.lc_dev + k, &m.lc_host[k], sizeof L, hipMemcpyHostToDevice, m.stream));
  m.lc_valid[k] = true;
  return m.lc_dev + k;
}

// Tail phase clocks of the last FX_TRACE_N fused exchanges (HF2D_FX_SKIP bit
// 4 on a loopback run): FX_TRACE_W words per step, zero where none ran.
std::vector<unsigned long long> DeviceSolver::fx_trace() {
  flush_pending();
  Impl& m = *impl;
  std::vector<unsigned long long> v((size_t)FX_TRACE_N * FX_TRACE_W, 0ull);
  if (!m.p2p.done) return v;
  HIP_CHECK(hipStreamSynchronize(m.stream));
  HIP_CHECK(hipMemcpy(v.data(), m.p2p.done + (DT_SHARDS + 1) * FX_DONE_STRIDE, v.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
  return v;
}

FusedX DeviceSolver::fused_args() const {
  const Impl& m = *impl;
  const Impl::P2P& p = m.p2p;
  const bool has_left = gi0 > 0, has_right = gi1 < cs.J.nx;
  FusedX X{};
  X.peer_recv_l = has_left ? p.push_base(0, m.rank, m.halo_cap) : nullptr;
  X.peer_recv_r = has_right ? p.push_base(1, m.rank, m.halo_cap) : nullptr;
  X.my_recv = (const real*)(p.base + p.off_recv);
  X.peer_flags = p.d_flags;
  X.peer_dtr = p.d_dtr;
  X.my_flags = (const unsigned long long*)p.base;
  X.my_dtr = (const double*)(p.base + p.off_dtr);
  X.seq = p.seq;
  X.done = p.done;
  X.cap = m.halo_cap;
  X.rank = m.rank;
  X.nranks = m.nranks;
  X.sides = (has_left ? 1 : 0) | (has_right ? 2 : 0);
  X.on = 1;
  static const int skip = std::getenv("HF2D_FX_SKIP") ? std::atoi(std::getenv("HF2D_FX_SKIP")) : 0;
  X.skip = m.p2p.loop ? skip : 0;   // (loopback timing runs only)
  static const int ef = std::getenv("HF2D_FX_EDGE_FIRST") ? std::atoi(std::getenv("HF2D_FX_EDGE_FIRST")) : 0;
  static const int c1 = std::getenv("HF2D_FX_COUNT1") ? std::atoi(std::getenv("HF2D_FX_COUNT1")) : 0;
  X.edge_first = ef;
  X.count1 = c1;
  return X;
}

// After fused-exchange steps the newest ghost columns and the peers' dt live
// only in the mailbox: materialise them before any other consumer.
void DeviceSolver::p2p_complete(bool keep_lns) {
  Impl& m = *impl;
  if (lns_ghost_pending && !keep_lns) {
    // the last fused lean N-S / mechanism step's halo: mailbox -> ghost columns
    lns_ghost_pending = false;
    const ColList& Lc = m.lns_pend;
    const int cnt = Lc.nf * h.ny;
    hipLaunchKernelGGL(hf2d_p2p_unpack, dim3((unsigned)std::max(1, std::min((2 * cnt + BLOCK - 1) / BLOCK, 1024))),
                       dim3(BLOCK), 0, m.stream, Lc, l_off - 1, l_off + (gi1 - gi0), h.ny, cnt, fused_args());
    HIP_CHECK(hipGetLastError());
  }
  if (!fx_pending) return;
  fx_pending = false;
  const long N = h.N;
  ColList L;
  L.nf = 0;
  const bool sg = lean_sg && lean_sg_ok;
  for (int k = 0; k < (sg ? 4 : 4 + NCOMP); k++) L.f[L.nf++] = m.S[sbuf] + (long)k * N;
  if (!sg)
    for (int k = 0; k < NCOMP; k++) L.f[L.nf++] = m.Spre[pbuf] + (long)k * N;
  L.f[L.nf++] = m.U[pbuf];
  L.f[L.nf++] = m.V[pbuf];
  L.f[L.nf++] = m.P2[pbuf];
  hipLaunchKernelGGL(hf2d_p2p_complete, dim3(1), dim3(P2P_THREADS), 0, m.stream, L, l_off - 1, l_off + (gi1 - gi0), h.ny,
                     L.nf * h.ny,
                     fused_args(), m.sc, (int)(nstep % 3));
  HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Step graphs.  Plain steps (no residual pass, no host read-back) are queued
// and executed GRAPH_STEPS at a time as one captured hipGraph: every kernel
// argument is step-invariant over that window (dt, time and the scenario
// CFL/beta come from device memory; ping-pong parities repeat every 2 steps
// and dt slots every 3, so 6 steps bring both back), which removes the
// per-launch host cost that dominates small multi-GPU strips.  Any capture
// error disables graphs for the solver and the queue runs eagerly.
// ---------------------------------------------------------------------------
namespace {
constexpr int GRAPH_STEPS = 6;
// Everything that selects the kernels of a step besides the step parameters
// (DeviceSolver::mode_signature): a window replays only under the same one.
uint64_t graph_signature(const StepParams& P, uint64_t mode) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
  mix((uint64_t)P.fpa.is_mu_t);
  mix((uint64_t)P.fpa.is_init);
  mix((uint64_t)P.fpa.isSrcAdd);
  mix(mode);
  return h;
}
}  // namespace

struct DeviceSolver::GraphCache {
  hipGraphExec_t exec = nullptr;
  uint64_t sig = 0;
  // fused lean N-S windows: the first step unpacks the previous step's halo
  // in its prologue (needs the mailbox to hold an lns list's publication at
  // replay), and the window ends with its last step's halo pending
  bool lns_pro = false, lns_end = false;
  ColList lns_end_list{};
  ~GraphCache() {
    if (exec) (void)hipGraphExecDestroy(exec);
  }
};

void DeviceSolver::flush_pending() {
  if (pending.empty()) return;
  std::vector<StepParams> q;
  q.swap(pending);
  for (const StepParams& p : q) do_step_eager(p, false);
}

uint64_t DeviceSolver::mode_signature() const {
  // (the ping-pong parities too: a captured window bakes in the buffer
  // pointers of its first step, and a materialise + re-entry (split) step
  // flips only some of them, so a window cached before a download must not
  // replay after it -- it did, and the lean mechanism run then stepped on
  // the previous level's buffers from the first replayed window on)
  const int fields[] = {lean_state, (int)lean, (int)fused, (int)lean_tile, (int)(lean_sg && lean_sg_ok), lean_cpt,
                        lean_tj, lean_nt, lean_wgcu, (int)(p2p_fuse && impl->p2p.on), (int)(sgl && sgl_ok), lns_state,
                        (int)lean_ns, (int)lean_mech, sbuf, abuf, dsbuf, pbuf, cbuf};
  uint64_t h = 0;
  for (int f : fields) h = h * 1000003ull + (uint64_t)(f + 1);
  return h;
}

StepResult DeviceSolver::do_step(const StepParams& P0, bool want_res) {
  Impl& m = *impl;
  // (the in-process host transport synchronises on the host: eager only;
  // so does lnm_timing, which waits for each step's phase events)
  const bool plain = use_graph && !want_res && !step_outputs && !lnm_timing && (!m.local || m.p2p.on) &&
                     !(lean && lean_ok && lean_state == 0) &&
                     !(lns_state == 0 && lns_entry(P0));   // lean N-S entry step: eager
  if (!plain || (pending.empty() && nstep % GRAPH_STEPS != 0)) {
    flush_pending();
    return do_step_eager(P0, want_res);
  }
  pending.push_back(P0);
  if ((int)pending.size() == GRAPH_STEPS) run_graph();
  StepResult r;
  r.async = true;
  return r;
}

void DeviceSolver::run_graph() {
  Impl& m = *impl;
  m.sc_mirrored = false;
  const uint64_t mode = mode_signature();
  const uint64_t sig = graph_signature(pending[0], mode);
  bool same = true;
  for (const StepParams& p : pending) same = same && graph_signature(p, mode) == sig;
  if (!same) {
    flush_pending();
    return;
  }
  if (!graph) graph.reset(new GraphCache);
  if (graph->exec && graph->sig == sig) {
    if (graph->lns_pro && !lns_last_valid) {   // (the mailbox holds another exchange's layout)
      flush_pending();
      return;
    }
    if (!graph->lns_pro) p2p_complete();
    HIP_CHECK(hipGraphLaunch(graph->exec, m.stream));
    if (graph->lns_end) {
      m.lns_pend = graph->lns_end_list;
      lns_ghost_pending = lns_last_valid = true;
    }
    dt_word_valid = false;   // (conservative: the next eager step reads the shards too)
    nstep += GRAPH_STEPS;   // ping-pong parities are unchanged after an even number of steps
    pending.clear();
    graph_launches++;
    return;
  }
  // capture the window (host bookkeeping advances as in eager mode)
  const long nstep0 = nstep;
  const int ab = abuf, ds = dsbuf, pb = pbuf, sb = sbuf, ls = lean_state;
  std::vector<StepParams> q;
  q.swap(pending);
  hipGraph_t g = nullptr;
  // (a replayed window may follow any launch: its first step reads the shards)
  dt_word_valid = false;
  const bool s_pend = lns_ghost_pending, s_valid = lns_last_valid;
  const ColList s_list = m.lns_pend;
  bool first_pro = false;
  bool ok = hipStreamBeginCapture(m.stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
  if (ok) {
    try {
      for (size_t k = 0; k < q.size(); k++) {
        lns_pro_uses = 0;
        do_step_eager(q[k], false);
        if (k == 0) first_pro = lns_pro_uses > 0;
      }
    } catch (const std::exception&) {
      ok = false;
    }
    hipGraph_t gg = nullptr;
    const bool ended = hipStreamEndCapture(m.stream, &gg) == hipSuccess;
    ok = ok && ended && gg != nullptr;
    if (gg && !ok) (void)hipGraphDestroy(gg);
    g = ok ? gg : nullptr;
  }
  hipGraphExec_t exec = nullptr;
  if (ok) ok = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) == hipSuccess;
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  // restore the bookkeeping and execute
  nstep = nstep0;
  abuf = ab;
  dsbuf = ds;
  pbuf = pb;
  sbuf = sb;
  lean_state = ls;
  if (!ok) {
    use_graph = false;   // eager from now on
    lns_ghost_pending = s_pend;   // (nothing of the capture ran)
    lns_last_valid = s_valid;
    m.lns_pend = s_list;
    for (const StepParams& p : q) do_step_eager(p, false);
    return;
  }
  if (graph->exec) (void)hipGraphExecDestroy(graph->exec);
  graph->exec = exec;
  graph->sig = sig;
  graph->lns_pro = first_pro;
  graph->lns_end = lns_ghost_pending && lns_last_valid;
  graph->lns_end_list = m.lns_pend;
  HIP_CHECK(hipGraphLaunch(graph->exec, m.stream));
  nstep += GRAPH_STEPS;
  graph_launches++;
}

// Split predict + fill step (every N-S / mechanism / generic case).
void DeviceSolver::step_split(const StepParams& P0, bool want_res, int slot, int slot_next, int serial, unsigned nblk,
                              bool to_lns) {
  StepParams P = P0;
  Impl& m = *impl;
  hipStream_t st = m.stream;
  const long c0 = (long)P.i0 * P.ny, c1 = (long)P.i1 * P.ny;
    SoA in = m.view(h, sbuf, abuf, dsbuf, pbuf);
    SoA mid = m.view(h, 1 - sbuf, abuf, 1 - dsbuf, pbuf);
    // single-gas N-S: only the live equations and fields move (SK_SGL/SK_SGT);
    // mechanism mode: SK_MECH (Euler and N-S)
    const int mode = m.mech ? SK_MECH : (P.sm == SM_NS && sgl) ? sk_mode : SK_GENERIC;
    // the ghost columns hold the lean N-S / mechanism representation (the
    // record was materialised): the split step's halo first
    if (ghost_stale) exchange(CpuSolver::HALO_STATE);
    // the ghost columns were last exchanged for a single-gas specialisation
    // and this step is generic (sgl switched off): refresh them in full first
    if (ghost_mode >= 0 && ghost_mode != SK_GENERIC && mode == SK_GENERIC)
      exchange(CpuSolver::HALO_STATE, -1, nullptr, true);
    // XCD-aware order: split Step 63.8 -> 59.2 us, resonator 117.7 -> 107.8 us
    // on 1x MI355X; the mechanism pair is 2 % slower with it (1.767 vs 1.800 ms)
    P.xcd = (split_xcd && (mode != SK_MECH || split_xcd_mech)) ? 1 : 0;
    hipLaunchKernelGGL(kPredict[want_res][mode], dim3(nblk), dim3(BLOCK), 0, st, P, in, mid, c0, c1, m.sc, slot,
                       slot_next, serial, m.partials);
    HIP_CHECK(hipGetLastError());
    const bool multi = (m.comm || m.local || m.p2p.on) && m.nranks > 1;
    if (P.sm == SM_NS) exchange(CpuSolver::HALO_MID);
    SoA sin = m.view(h, 1 - sbuf, abuf, 1 - dsbuf, pbuf);
    SoA out = m.view(h, sbuf, abuf, 1 - dsbuf, 1 - pbuf);
    if (to_lns && mode == SK_MECH) {
      // entering the lean mechanism path: transport of level n+1 into the
      // second buffers (level n stays for G_{n+1}); the state (T, p, Cp, k)
      // of level n+1 is read from the generic arrays (T copied to Tst[0])
      out.mu = m.mu2;
      out.lam = m.lam2;
      out.mu_t = m.mu_t2;
    } else if (to_lns) {   // entering the lean N-S path: level n+1 into the second buffers
      out.CP = m.CP2;
      out.mu = m.mu2;
      out.lam = m.lam2;
      out.kk = m.kk2;
      out.mu_t = m.mu_t2;
    }
    if (mode == SK_MECH) {
      // operator-split kinetics: Ys[1-sbuf] -> Ys[sbuf]; N-S strips also react
      // their ghost columns (exchanged above; same inputs as on the owner)
      const bool ghosts = multi && P.sm == SM_NS;
      const long k0 = ghosts ? c0 - (c0 > 0 ? h.ny : 0) : c0;
      const long k1 = ghosts ? c1 + (c1 < h.N ? h.ny : 0) : c1;
      const unsigned nbk = (unsigned)((k1 - k0 + BLOCK - 1) / BLOCK);
      launch_chem(P, sin, out, k0, k1, nbk, slot);
      m.mech_view(sin, sbuf, 1 - dsbuf);   // the fill reads the post-chemistry species
    }
    // SGL: gradients / Diff only when the host reads the record (or y+ follows)
    const int sg_out = (step_outputs || want_res) ? 1 : 0;
    // SGT / mechanism: the gradients an active N-S cell stores are recomputed
    // by its next fill before any use (fill_compute), so between outputs
    // (and the wall friction velocities of the cycle end, an output step) they
    // are dead stores: 80 B/cell (HF2D_GRAD_EVERY=1 stores them every step)
    const int tg_out = grad_every ? 1 : sg_out;
    // register budget: measured on 1x MI355X (tools/fill_occ_sweep.sh): the
    // mechanism fill is 10 % faster at 2 waves/SIMD (256 VGPRs, a few spills)
    // than at the compiler's 1; SGL / SGT are fastest at the default
    const int focc = fill_occ >= 0 ? fill_occ : (mode == SK_MECH ? 2 : 0);
    FillK fk;
    int store = 1;
    if (mode == SK_MECH) {
      store = tg_out;
      fk = m.nsp > 9 ? hf2d_fill<SK_MECH, MECH_MAXSP>
                     : (mech_lazy && focc == 2) ? hf2d_fill_occ<SK_MECH, 9, 2, true> : kFill[SK_MECH][occ_slot(focc)];
    } else {
      store = mode == SK_SGL ? sg_out : mode == SK_SGT ? tg_out : 1;
      fk = kFill[mode][mode == SK_GENERIC ? 0 : occ_slot(focc)];
    }
    hipLaunchKernelGGL(fk, dim3(nblk), dim3(BLOCK), 0, st, P, sin, sin, out, c0, c1, m.sc, slot, slot_next, serial,
                       store);
    HIP_CHECK(hipGetLastError());
    dsbuf = 1 - dsbuf;
    pbuf = 1 - pbuf;
}

bool DeviceSolver::lns_entry(const StepParams& P0) const {
  StepParams P = P0;
  P.ny = h.ny;
  return (lean_ns && lns_ok && lns_step_ok(P)) || (lean_mech && lnm_ok && lnm_step_ok(P));
}

// The lean mechanism step applies (lean_mech.hpp; eligibility lnm_ok) with a
// list-building kinetics kernel (compiled or hiprtc-specialised)
bool DeviceSolver::lnm_step_ok(const StepParams& P) const {
  const Impl& m = *impl;
  const int kind = chem_kernel ? chem_kernel : ((chem_fast && chem_fast_ok) ? 1 : (chem_rtc && chem_rtc_ok) ? 4 : 2);
  return lean_mech && lnm_ok && m.mech && P.sm == SM_NS && chem_compact &&
         ((kind == 1 && chem_fast_ok) || (kind == 4 && chem_rtc_ok)) && !P.fpa.is_init && !P.ffc.is_init &&
         P.fpa.is_mu_t == lns_prev_mu_t && P.ny >= LNM_TILE;
}

using LnmK = void (*)(StepParams, LnmArrays, LeanTile, DevScalars*, int, int, int, ResidualPack*);
// [residual][SST]
// [residual][SST][strip with a right neighbour] (residual steps: the strip variant)
static const LnmK kLnm[2][2][2] = {
    {{hf2d_lnm_step<false, 0, false>, hf2d_lnm_step<false, 0, true>},
     {hf2d_lnm_step<false, 3, false>, hf2d_lnm_step<false, 3, true>}},
    {{hf2d_lnm_step<true, 0>, hf2d_lnm_step<true, 0>}, {hf2d_lnm_step<true, 3>, hf2d_lnm_step<true, 3>}}};

// One lean mechanism step (lean_mech.hpp): tile kernel, kinetics of the
// listed cells in place on the new species, their state kernel.
std::vector<unsigned long long> DeviceSolver::lnm_trace_fetch() {
  synchronize();
  Impl& m = *impl;
  std::vector<unsigned long long> v((size_t)m.lnm_trace_n * 12);
  if (!v.empty()) HIP_CHECK(hipMemcpy(v.data(), m.lnm_trace, v.size() * 8, hipMemcpyDeviceToHost));
  return v;
}

void DeviceSolver::lnm_step(const StepParams& P, bool want_res, int slot, int slot_next, int serial) {
  Impl& m = *impl;
  hipStream_t st = m.stream;
  LnmArrays a = m.lnm_arrays(h, sbuf, pbuf, cbuf, dsbuf, abuf);
  if (std::getenv("HF2D_LNM_TRACE")) {   // phase trace of every step (the last one is kept)
    const long nwg = (long)((P.i1 - P.i0 + lnm_ti - 1) / lnm_ti) * ((P.ny + LNM_TILE - 1) / LNM_TILE);
    if (!m.lnm_trace || m.lnm_trace_n < nwg) {
      m.lnm_trace = m.mem.alloc<unsigned long long>(nwg * 12);
      m.lnm_trace_n = nwg;
    }
    a.tr = m.lnm_trace;
  }
  if (lnm_ti < 1 || lnm_ti > BLOCK / LNM_TILE) lnm_ti = BLOCK / LNM_TILE;
  LeanTile T = lnm_tile(P.i1 - P.i0, P.ny, lnm_ti);
  T.ne = (P.i1 - P.i0) % T.TI == 1 ? 2 : 1;   // (the halo's second column from the edge part)
  // RCCL / in-process transports: the tiles of the strip's first and last
  // tile columns first -- with their kinetics and state kernel, which change
  // the reacting edge cells' halo values -- then their halo on the comm
  // stream while the interior tiles and their kinetics run (a second list),
  // then the dt MIN (as the lean N-S and inviscid tile kernels)
  // (the decision must be the same on every rank -- the exchange sequence
  // differs -- so a strip too narrow to split runs all its tiles at once)
  // Opt-in (lnm_overlap / HF2D_LNM_SPLIT=1): the edge part is one
  // workgroup round of ~50 tiles on an otherwise idle GPU before the interior
  // starts, so on the mailbox transport the split step measured 109 us of
  // exchange cost against 17 us for all tiles + push / unpack
  // (tools/exchange_loopback.py, scramjet 8 ranks, profiles/exchange_loopback_r05.md)
  static const bool split_env = std::getenv("HF2D_LNM_SPLIT") && std::string(std::getenv("HF2D_LNM_SPLIT")) == "1";
  lnm_split = (split_env || lnm_overlap) && comm_overlap && (m.p2p.on ? p2p_fuse : (m.comm || m.local)) && m.nranks > 1 &&
              !want_res && cs.cfg.isAdiabaticWall;
  const bool parts = T.nbi >= 2 + T.ne;
  // (xGMI mailboxes: the edge halo is pushed before the interior tiles run,
  // and published with the dt once they are done)
  ColList Lc{};
  if (lnm_split && m.p2p.on) {
    sbuf = 1 - sbuf, pbuf = 1 - pbuf, cbuf = 1 - cbuf, dsbuf = 1 - dsbuf;
    std::vector<real*> fl;
    std::vector<unsigned char> fo;
    halo_fields(CpuSolver::HALO_LNS, fl, fo, false);
    sbuf = 1 - sbuf, pbuf = 1 - pbuf, cbuf = 1 - cbuf, dsbuf = 1 - dsbuf;
    if (fl.size() > (size_t)MAX_HALO_FIELDS || (long)fl.size() * h.ny > m.halo_cap)
      throw std::runtime_error("mechanism halo exceeds the mailbox capacity");
    Lc.nf = (int)fl.size();
    for (int k = 0; k < Lc.nf; k++) {
      Lc.f[k] = fl[k];
      Lc.o[k] = fo[k];
    }
  }
  if (!lnm_split) {
    a.hot = m.chem_list;
    a.hot_n = &m.sc->hot_cnt[slot];
    a.part = 0;
    // mailboxes: the previous step's halo (pushed after its state kernel,
    // exchange()) is unpacked by this step's edge tiles (fx_ghost_prologue)
    if (m.p2p.on && p2p_fuse && m.nranks > 1 && lns_prev_valid && lns_ghost_prologue) {
      a.lg = lc_device(m.lns_pend);
      if (a.lg) {
        a.xg = fx_device(fused_args());
        lns_ghost_pending = false;
        lns_pro_uses++;
        lns_prologue_steps++;
      }
    }
    p2p_complete();
    lnm_launch(P, a, T, want_res, slot, slot_next, serial, (unsigned)(T.nbi * T.nbj));
  } else {
    p2p_complete();
    if (!m.comm_stream) {
      HIP_CHECK(hipStreamCreateWithFlags(&m.comm_stream, hipStreamNonBlocking));
      HIP_CHECK(hipEventCreateWithFlags(&m.ev_edge, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&m.ev_halo, hipEventDisableTiming));
    }
    // edge list first (at most its own cells), the interior list after it:
    // tile column 0 (TI columns), ne - 1 full columns and the last, partial
    // one of w - (nbi - 1) TI columns -- the list holds exactly N entries
    const long wl = (long)(P.i1 - P.i0) - (long)(T.nbi - 1) * T.TI;
    const long edge_cells = ((long)T.ne * T.TI + wl) * P.ny;
    a.hot = m.chem_list;
    a.hot_n = &m.sc->hot_cnt[slot];
    a.part = parts ? 1 : 0;
    lnm_launch(P, a, T, want_res, slot, slot_next, serial, (unsigned)(parts ? (1 + T.ne) * T.nbj : T.nbi * T.nbj));
    const int cnt = Lc.nf * h.ny;
    if (m.p2p.on) {
      hipLaunchKernelGGL(push_kernel(push_per), dim3(push_grid(push_per, cnt)), dim3(BLOCK), 0, st, Lc, l_off, l_off + (gi1 - gi0) - 1, h.ny, cnt, fused_args(), m.sc, slot_next,
                         1, 0);
      HIP_CHECK(hipGetLastError());
    } else {
      HIP_CHECK(hipEventRecord(m.ev_edge, st));
    }
    a.hot = m.chem_list + edge_cells;
    a.hot_n = &m.sc->hot_cnt2[slot];
    a.part = 2;
    if (parts) lnm_launch(P, a, T, want_res, slot, slot_next, serial, (unsigned)((T.nbi - 1 - T.ne) * T.nbj));
    if (m.p2p.on) {
      hipLaunchKernelGGL(hf2d_p2p_finish, dim3(1), dim3(WAVE), 0, st, fused_args(), m.sc, slot_next);
      HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(hf2d_p2p_unpack, dim3((unsigned)std::max(1, std::min((2 * cnt + BLOCK - 1) / BLOCK, 1024))),
                         dim3(BLOCK), 0, st, Lc, l_off - 1, l_off + (gi1 - gi0), h.ny, cnt, fused_args());
      HIP_CHECK(hipGetLastError());
      ghost_stale = true;
      p2p_mwg_exchanges++;
      overlap_steps++;
    }
  }
  sbuf = 1 - sbuf;
  pbuf = 1 - pbuf;
  cbuf = 1 - cbuf;
  dsbuf = 1 - dsbuf;
  lnm_steps++;
  if (lnm_split && !m.p2p.on) {   // the new state's halo (post-step buffers), overlapped with the interior
    if (m.local) {   // in-process group: the host orders the streams (see the inviscid path)
      HIP_CHECK(hipEventSynchronize(m.ev_edge));
      exchange(CpuSolver::HALO_LNS, -1, (void*)m.comm_stream);
      HIP_CHECK(hipStreamSynchronize(m.comm_stream));
    } else {
      HIP_CHECK(hipStreamWaitEvent(m.comm_stream, m.ev_edge, 0));
      exchange(CpuSolver::HALO_LNS, -1, (void*)m.comm_stream);
      HIP_CHECK(hipEventRecord(m.ev_halo, m.comm_stream));
      HIP_CHECK(hipStreamWaitEvent(st, m.ev_halo, 0));
    }
    exchange_dt(slot_next);
    overlap_steps++;
  }
}

// Tile kernel (the tiles of a.part), kinetics of the cells it listed (a.hot /
// a.hot_n) in place on the new species, their state kernel.
void DeviceSolver::lnm_launch(const StepParams& P, const LnmArrays& a, const LeanTile& T, bool want_res, int slot,
                              int slot_next, int serial, unsigned ntile) {
  Impl& m = *impl;
  hipStream_t st = m.stream;
  const LnmLayout L(T.TI, T.TJ, m.nsp - 1);
  const size_t shmem = (size_t)L.total() * sizeof(real);
  const int strip = P.i1 < P.nx ? 1 : 0;
  const LnmK k = kLnm[want_res ? 1 : 0][lnm_turb == 3 ? 1 : 0][strip];
  // the dynamic-LDS limit is a property of the kernel function, shared by
  // every solver of the process (virtual ranks run on threads): raise it to
  // the largest layout asked for so far (tile width / species count vary)
  static std::atomic<int> attr_bytes[2][2][2] = {};
  static std::mutex attr_mu;
  std::atomic<int>& ab = attr_bytes[want_res ? 1 : 0][lnm_turb == 3 ? 1 : 0][strip];
  if (ab.load(std::memory_order_acquire) < (int)shmem) {
    std::lock_guard<std::mutex> lk(attr_mu);
    if (ab.load(std::memory_order_relaxed) < (int)shmem) {
      HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
      ab.store((int)shmem, std::memory_order_release);
    }
  }
  // lnm_timing: events around the three phases (measurement only: the host
  // waits for each step's events, so the steps serialise with the host)
  if (lnm_timing) {
    if (!m.lnm_ev[0])
      for (auto& e : m.lnm_ev) HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(m.lnm_ev[0], st));
  }
  hipLaunchKernelGGL(k, dim3(ntile), dim3(BLOCK), shmem, st, P, a, T, m.sc, slot, slot_next, serial, m.partials);
  HIP_CHECK(hipGetLastError());
  if (lnm_timing) HIP_CHECK(hipEventRecord(m.lnm_ev[1], st));
  // kinetics of the listed cells (T^m >= Tchem), in place on the new species
  const MechData& md = *cs.cfg.mech->data_ptr();
  SoA mid;
  mid.nx = h.nx;
  mid.ny = h.ny;
  mid.N = h.N;
  mid.S = a.Sp_out;
  mid.Ys = a.Ys_out;
  mid.CT = m.CT;
  mid.mech = m.mech;
  mid.nsp = m.nsp;
  const long c0 = (long)P.i0 * P.ny, c1 = (long)P.i1 * P.ny;
  const int kind = chem_kernel ? chem_kernel : ((chem_fast && chem_fast_ok) ? 1 : 4);
#ifdef HF2D_FP32
  (void)kind, (void)c0, (void)c1, (void)md;
  throw std::runtime_error("FP32 build: finite-rate kinetics need the FP64 build");
#else
  if (kind == 1) {
    if (!chem_fast_launch(cs.cfg.mech->name, P, mid, mid, a.To, c0, c1, m.sc, slot, md.Tchem, md.nsub, st, a.hot,
                          a.hot_n, true))
      throw std::runtime_error("hf2d_chem_fast list launch failed");
    chem_kernel_used = "hf2d_chem_fast";
  } else {
    if (!chem_rtc_launch(md, mid, mid, a.To, c0, c1, m.sc, slot, md.Tchem, md.nsub, st, a.hot, a.hot_n, true))
      throw std::runtime_error("hf2d_rtc_chem list launch failed");
    chem_kernel_used = "hf2d_rtc_chem";
  }
#endif
  if (lnm_timing) HIP_CHECK(hipEventRecord(m.lnm_ev[2], st));
  const unsigned nb = (unsigned)std::min<long>((c1 - c0 + BLOCK - 1) / BLOCK, 1024);
  hipLaunchKernelGGL(hf2d_lnm_hot, dim3(nb), dim3(BLOCK), 0, st, P, a, m.sc, slot, slot_next, serial);
  HIP_CHECK(hipGetLastError());
  if (lnm_timing) {
    HIP_CHECK(hipEventRecord(m.lnm_ev[3], st));
    HIP_CHECK(hipEventSynchronize(m.lnm_ev[3]));
    for (int q = 0; q < 3; q++) {
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, m.lnm_ev[q], m.lnm_ev[q + 1]));
      lnm_phase_ms[q] += ms;
    }
    lnm_phase_ms[3] += 1.0;
  }
}

// The lean N-S kernel applies to this step (lean_ns.hpp; eligibility lns_ok)
bool DeviceSolver::lns_step_ok(const StepParams& P) const {
  const Impl& m = *impl;
  // (the fill F_m runs in step m here but in step m-1 in the split stepper:
  // the step parameters it reads must agree, i.e. is_mu_t must not change)
  return lean_ns && lns_ok && P.sm == SM_NS && sgl && sgl_ok && (sk_mode == SK_SGL || sk_mode == SK_SGT) &&
         !m.mech && !P.fpa.is_init && !P.ffc.is_init &&
         P.fpa.is_mu_t == lns_prev_mu_t && P.ny >= LEAN_TILE_MIN_TJ;
}

StepResult DeviceSolver::do_step_eager(const StepParams& P0, bool want_res) {
  Impl& m = *impl;
  m.sc_mirrored = false;
  StepParams P = P0;
  P.nx = h.nx;
  P.ny = h.ny;
  P.i0 = l_off;
  P.i1 = l_off + (gi1 - gi0);
  P.gx0 = gi0 - l_off;
  P.do_residual = want_res ? 1 : 0;
  P.species = m.species;
  P.scen = m.scen;
  const long c0 = (long)P.i0 * P.ny, c1 = (long)P.i1 * P.ny;
  const unsigned nblk = (unsigned)((c1 - c0 + BLOCK - 1) / BLOCK);
  const int slot = nstep % 3, slot_next = (nstep + 1) % 3;
  const int serial = cs.cfg.semantics == Semantics::SERIAL ? 1 : 0;
  const bool euler = P.sm != SM_NS;
  hipStream_t st = m.stream;
  unsigned nres = nblk;   // workgroups that wrote residual partials
  int nres_waves = BLOCK / WAVE;   // ... and partials per workgroup
  const bool sg_now = lean_sg && lean_sg_ok;
  fx_step = false;
  // the slot's word holds the MIN only right after a folding tile launch
  const bool dt_word_ok = dt_word_valid;
  dt_word_valid = false;
  // the mailbox holds a fused lean N-S step's halo (list m.lns_pend) only
  // right after such a step (every other step or exchange publishes another
  // layout or nothing)
  lns_prev_valid = lns_last_valid;
  lns_last_valid = false;
  const bool tile_path = euler && lean && lean_ok && lean_tile &&
                         lean_state == 1 && P.ny >= LEAN_TILE_MIN_TJ;
  // (a fused lean N-S step unpacks the previous fused step's halo itself)
  const bool lns_fx_next = !euler && (lnm_step_ok(P) || lns_step_ok(P)) && lns_state == 1 && lean_state == 0 &&
                           m.p2p.on && p2p_fuse && m.nranks > 1;
  if (!tile_path) p2p_complete(lns_fx_next);
  if (euler && lean && lean_ok && lean_tile && lean_state == 1 && P.ny >= LEAN_TILE_MIN_TJ) {
    LeanSoA L = m.lean_view(h, sbuf, abuf, dsbuf, pbuf, false);
    P.skip_same = tile_skip_same ? 1 : 0;
    P.dt_read = dt_read_mode == 1 ? 1 : 0;
    // two cells per thread unless that leaves fewer than ~2 workgroups per CU
    // (small strips of a multi-GPU run)
    // (256-thread tiles only: the small-workgroup geometries are explicit
    // choices of the autotune)
    const bool sg = lean_sg && lean_sg_ok;
    const int nt = tile_nt(lean_nt, sg), nts = nt == 128 ? 0 : 1;
    int cpt = lean_cpt == 2 ? 2 : 1;
    if (cpt == 2 && nt == BLOCK) {
      const LeanTile T2 = lean_tile_geom(P.i1 - P.i0, P.ny, BLOCK, lean_tj, 2);
      if ((long)T2.nbi * T2.nbj < 2L * cu_count) cpt = 1;
    }
    const LeanTile T = lean_tile_geom(P.i1 - P.i0, P.ny, nt, lean_tj, cpt);
    const unsigned ntile = (unsigned)(T.nbi * T.nbj);
    size_t shmem = (size_t)lean_tile_fields(sg) * T.NC * sizeof(real);
    if (lean_wgcu > 0)   // cap the resident workgroups per CU through the LDS request (160 KB per CU)
      shmem = std::max(shmem, (size_t)((LDS_PER_CU / lean_wgcu - 1024) & ~255));
    const bool out = step_outputs || want_res;
    // staggered start only for a grid that is resident at once (<= 4 dispatch
    // rounds: measured 1.5 us faster on the headline grid; the 4000x1000 triple
    // point, dispatched in ~15 waves, ran 350 -> 550 us with it)
    P.stagger_wgs = cu_count > 0 ? cu_count : 256;
    P.stagger = ntile <= 4u * (unsigned)P.stagger_wgs && nt == BLOCK ? tile_stagger : 0;
    // (64-thread tiles, the whole grid resident at once: a linear start ramp
    // over the grid of 2 / 4 / 7 / 10 us measured 4.7 / 6.4 / 15 / 27 %
    // slower than none, profiles/r04_start.md)
    // multi-GPU: exchange fused into the tile kernel (no separate exchange launch)
    fx_step = m.p2p.on && p2p_fuse && !lean_has_cauchy_x;
    FusedX X = fx_step ? fused_args() : FusedX{};
    // lagged dt: the fused tail waits for the two neighbours only; the dt
    // MIN follows in the next fused step's first workgroup or in
    // hf2d_p2p_complete before any other consumer (fx_pending)
    X.defer = fx_step && P.lag_dt ? 1 : 0;
    // RCCL / in-process transports: edge tiles first, their halo on the comm
    // stream while the interior tiles compute, then the dt MIN
    // (the decision must be the same on every rank -- the exchange sequence
    // differs -- so a strip too narrow to split runs all its tiles at once)
    const bool split = comm_overlap && !fx_step && !m.p2p.on && (m.comm || m.local) && m.nranks > 1 &&
                       !want_res && !out && !tile_trace && lean_occ == 0;
    if (split) {
      if (!m.comm_stream) {
        HIP_CHECK(hipStreamCreateWithFlags(&m.comm_stream, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&m.ev_edge, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&m.ev_halo, hipEventDisableTiming));
      }
      const bool parts = T.nbi >= 3;
      const unsigned ne = parts ? (unsigned)(2 * T.nbj) : ntile, ni = parts ? (unsigned)((T.nbi - 2) * T.nbj) : 0u;
      const TileK pk = nt == BLOCK ? kTile[sg][cpt - 1][0] : kTileNt[nts][cpt - 1][0];
      hipLaunchKernelGGL(pk, dim3(ne), dim3(nt), shmem, st, P, L, T, m.sc, slot, slot_next, serial, m.partials,
                         parts ? 1 : 0);
      HIP_CHECK(hipGetLastError());
      sbuf = 1 - sbuf;   // the new state is this step's output arrays
      dsbuf = 1 - dsbuf;
      pbuf = 1 - pbuf;
      HIP_CHECK(hipEventRecord(m.ev_edge, st));
      // interior tiles in flight before the (possibly host-blocking) exchange
      // is issued; they write neither the edge columns nor the ghost columns
      if (ni > 0)
        hipLaunchKernelGGL(pk, dim3(ni), dim3(nt), shmem, st, P, L, T, m.sc, slot, slot_next, serial, m.partials,
                           2);
      HIP_CHECK(hipGetLastError());
      if (m.local) {
        // in-process group: the host orders the two streams (waits on it).
        // Device-side cross-stream waits would put barrier packets in hardware
        // queues that several virtual ranks' streams share, and a wait cycle
        // across those queues can deadlock.
        HIP_CHECK(hipEventSynchronize(m.ev_edge));
        exchange(CpuSolver::HALO_LEAN, -1, (void*)m.comm_stream);
        HIP_CHECK(hipStreamSynchronize(m.comm_stream));
      } else {
        HIP_CHECK(hipStreamWaitEvent(m.comm_stream, m.ev_edge, 0));
        exchange(CpuSolver::HALO_LEAN, -1, (void*)m.comm_stream);
        HIP_CHECK(hipEventRecord(m.ev_halo, m.comm_stream));
        HIP_CHECK(hipStreamWaitEvent(st, m.ev_halo, 0));
      }
      exchange_dt(slot_next);
      overlap_steps++;
      nstep++;
      StepResult r;
      r.async = true;
      return r;
    }
    // variant: 0 plain, 1 outputs, 2 residual (all variants of one step use
    // the cpt the tile geometry was built for)
    const int var = want_res ? 2 : out ? 1 : 0;
    if (tile_trace && var == 0 && !fx_step)
      hipLaunchKernelGGL(nt == BLOCK ? kTileTr[sg][cpt - 1] : kTileTrNt[nts][cpt - 1], dim3(ntile), dim3(nt), shmem,
                         st, P, L, T, m.sc, slot, slot_next, serial, m.partials, tile_trace);
    else if (fx_step) {
      // the fused tail folds every rank's dt into the next slot's word
      // (fx_tail): the next fused step reads that one word (not when the
      // fold is deferred, lagged dt)
      const bool word = dt_read_mode >= 1 && !X.defer;
      if (word && dt_word_ok) P.dt_read = 2;
      hipLaunchKernelGGL(nt == BLOCK ? kTileFx[sg][cpt - 1][var] : kTileFxNt[nts][cpt - 1][var], dim3(ntile),
                         dim3(nt), shmem, st, P, L, T, m.sc, slot, slot_next, serial, m.partials, fx_device(X));
      dt_word_valid = word;
    } else if (sg && cpt == 1 && var == 0 && lean_occ == 6 && !tile_trace && nt == BLOCK)
      hipLaunchKernelGGL((hf2d_lean_tile_occ<false, false, true, 6>), dim3(ntile), dim3(BLOCK), shmem, st, P, L, T,
                         m.sc, slot, slot_next, serial, m.partials);
    // (multi-gas, one cell per thread, at a 5-wave register budget -- 96
    // VGPRs + 10 spilled instead of 103: the triple point ran 351 -> 365 us)
    else {
      // single GPU, last step of the host call: the scalars go to the host
      // mirror from the kernel's own tail (host_tail)
      const bool mirror = var == 1 && !tile_trace && host_tail && m.nranks == 1 && !m.local && !m.p2p.on;
      if (mirror) {
        P.host_sc = m.sc_host;
        P.host_done = m.host_done;
      }
      // dt read of the tile kernel (StepParams::dt_read): with dt_read_mode
      // 2 every step's last workgroup folds the shards into the word and the
      // next step's workgroups read that one word
      const bool fold = dt_read_mode == 2 && !tile_trace && m.nranks == 1 && !m.local && !m.p2p.on;
      P.dt_read = (fold && dt_word_ok) ? 2 : dt_read_mode == 1 ? 1 : 0;
      if (fold) {
        P.dt_fold = 1;
        P.host_done = m.host_done;
      }
      if (nt != BLOCK)
        hipLaunchKernelGGL(kTileNt[nts][cpt - 1][var], dim3(ntile), dim3(nt), shmem, st, P, L, T, m.sc, slot,
                           slot_next, serial, m.partials, 0);
      else
        hipLaunchKernelGGL(kTile[sg][cpt - 1][var], dim3(ntile), dim3(BLOCK), shmem, st, P, L, T, m.sc, slot,
                           slot_next, serial, m.partials, 0);
      m.sc_mirrored = mirror;
      dt_word_valid = fold;
    }
    HIP_CHECK(hipGetLastError());
    nres = ntile;
    nres_waves = nt / WAVE;
    sbuf = 1 - sbuf;
    dsbuf = 1 - dsbuf;
    pbuf = 1 - pbuf;
  } else if (euler && lean && lean_ok) {
    const bool fromg = lean_state == 0;
    LeanSoA L = m.lean_view(h, sbuf, abuf, dsbuf, pbuf, fromg);
    hipLaunchKernelGGL(kLeanEuler[want_res][fromg], dim3(nblk), dim3(BLOCK), 0, st, P, L, c0, c1, m.sc, slot,
                       slot_next, serial, m.partials);
    HIP_CHECK(hipGetLastError());
    sbuf = 1 - sbuf;
    dsbuf = 1 - dsbuf;
    pbuf = 1 - pbuf;
    lean_state = 1;
  } else if (euler && fused && !m.mech) {
    if (lean_state) lean_materialize();
    // Predictor and fill of a cell run back to back in one thread, so the
    // new state goes to the other S buffer (neighbours still read the old
    // one) and the current-state index flips.
    SoA in = m.view(h, sbuf, abuf, dsbuf, pbuf);
    SoA mid = m.view(h, 1 - sbuf, abuf, 1 - dsbuf, pbuf);
    SoA out = m.view(h, 1 - sbuf, 1 - abuf, 1 - dsbuf, pbuf);
    hipLaunchKernelGGL(want_res ? hf2d_fused_euler<true> : hf2d_fused_euler<false>, dim3(nblk), dim3(BLOCK), 0, st,
                       P, in, mid, out, c0, c1, m.sc, slot, slot_next, serial, m.partials);
    HIP_CHECK(hipGetLastError());
    abuf = 1 - abuf;
    dsbuf = 1 - dsbuf;
    sbuf = 1 - sbuf;
  } else if (lnm_step_ok(P)) {
    if (lean_state) lean_materialize();
    if (lns_state == 0) {
      // first lean mechanism step: the split step, then T^{n+1} as the stored state.
      // Its fill F_{n+1} overwrites the level-n state (Cp, k, p) in place; a
      // materialise right after this step (a download after a one-step call)
      // re-runs F_{n+1}, which reads the lagged state from the [cbuf] buffers
      // as after a lean step: keep level n there (without it the re-fill read
      // stale buffers: with a download after every step the scramjet's dt
      // left the CPU stepper's at step 4; test_download_after_every_step_leaves_the_trajectory_unchanged)
      const size_t SB = (size_t)h.N * sizeof(real);
      HIP_CHECK(hipMemcpyAsync(m.CP2, m.CP, SB, hipMemcpyDeviceToDevice, st));
      HIP_CHECK(hipMemcpyAsync(m.kk2, m.kk, SB, hipMemcpyDeviceToDevice, st));
      HIP_CHECK(hipMemcpyAsync(m.p2, m.p, SB, hipMemcpyDeviceToDevice, st));
      step_split(P, want_res, slot, slot_next, serial, nblk, true);
      HIP_CHECK(hipMemcpyAsync(m.Tst[0], m.Tg[pbuf], h.N * sizeof(real), hipMemcpyDeviceToDevice, st));
      lns_state = 1;
      cbuf = 1;
    } else {
      lnm_step(P, want_res, slot, slot_next, serial);
      const LeanTile T = lnm_tile(P.i1 - P.i0, P.ny, lnm_ti);
      nres = (unsigned)(T.nbi * T.nbj);
    }
  } else if (lns_step_ok(P)) {
    if (lean_state) lean_materialize();
    if (lns_state == 0) {
      // first lean N-S step: the split step with the fill's CP/mu/lam/k going
      // to the second level buffers (the level it read stays for K_{n+1})
      step_split(P, want_res, slot, slot_next, serial, nblk, true);
      lns_state = 1;
      cbuf = 1;
    } else {
      const LnsArrays a = m.lns_arrays(h, sbuf, pbuf, cbuf, dsbuf, abuf);
      LeanTile T = lean_tile_geom(P.i1 - P.i0, P.ny, BLOCK, lean_tj > 0 ? lean_tj : lns_tile_height(P.ny, BLOCK), 1);
      // (the halo's second column must come from the edge part)
      T.ne = (P.i1 - P.i0) % T.TI == 1 ? 2 : 1;
      const int ntile = T.nbi * T.nbj;
      const bool t2 = sk_mode == SK_SGT;
      const size_t shmem = (size_t)(t2 ? Lns<SK_SGT>::PLANES : Lns<SK_SGL>::PLANES) * T.NC * sizeof(real);
      // register budget (measured, 1x MI355X): the k-eps kernel compiles to
      // ~173 VGPRs (2 waves/SIMD); a 3-wave budget is 11 % faster (resonator
      // 2000x200: 110.7 -> 98.8 us/step); the laminar one is best unbounded
      const int occ = lns_occ > 0 ? lns_occ : (t2 ? 3 : 0);
      // (a residual step runs the compiler's register budget)
      const int tv = !t2 ? 0 : lns_turb == 3 ? 2 : lns_turb == 4 ? 3 : 1;
      const LnsK lk = kLns[tv][want_res][want_res ? 0 : (occ == 5 ? 2 : occ == 3 ? 1 : 0)];
      // xGMI mailboxes: the exchange fused into the tile kernel (edge cells
      // push their HALO_LNS values to the neighbour, the last workgroup
      // publishes the step and folds the peers' dt), then one unpack kernel;
      // RCCL / in-process transports: edge tiles first, their halo on the comm
      // stream while the interior tiles compute, then the dt MIN (as the
      // inviscid tile kernel)
      ColList Lc{};
      lns_fx = m.p2p.on && p2p_fuse && m.nranks > 1;
      if (lns_fx) {   // the HALO_LNS pointers of the post-step buffers
        sbuf = 1 - sbuf, pbuf = 1 - pbuf, cbuf = 1 - cbuf, dsbuf = 1 - dsbuf;
        std::vector<real*> fl;
        std::vector<unsigned char> fo;
        halo_fields(CpuSolver::HALO_LNS, fl, fo, false);
        sbuf = 1 - sbuf, pbuf = 1 - pbuf, cbuf = 1 - cbuf, dsbuf = 1 - dsbuf;
        if (fl.size() > (size_t)MAX_HALO_FIELDS || (long)fl.size() * h.ny > m.halo_cap)
          throw std::runtime_error("lean N-S halo exceeds the mailbox capacity");
        Lc.nf = (int)fl.size();
        for (int k = 0; k < Lc.nf; k++) {
          Lc.f[k] = fl[k];
          Lc.o[k] = fo[k];
        }
      }
      // (the decision must be the same on every rank -- the exchange sequence
      // differs -- so a strip too narrow to split runs all its tiles at once)
      lns_split = !lns_fx && comm_overlap && !m.p2p.on && (m.comm || m.local) && m.nranks > 1 && !want_res &&
                  cs.cfg.isAdiabaticWall;
      const bool lparts = T.nbi >= 2 + T.ne;
      if (lns_fx) {
        // the previous fused step's halo is still in the mailbox: this
        // kernel's edge tiles copy it into the ghost columns they read
        // (fx_ghost_prologue) instead of a separate unpack launch
        // (valid whenever the mailbox's last publication was a fused lean
        // N-S step: its parity stays untouched until this step publishes,
        // so the copy is exact even if p2p_complete already unpacked it)
        const ColList* Lg = nullptr;
        if (lns_prev_valid && lns_ghost_prologue) {
          Lg = lc_device(m.lns_pend);
          if (Lg) {
            lns_ghost_pending = false;
            lns_pro_uses++;
            lns_prologue_steps++;
          }
        }
        p2p_complete();   // (a list new inside a capture: the separate unpack)
        hipLaunchKernelGGL(kLnsFx[tv][want_res ? 1 : 0], dim3(ntile), dim3(BLOCK), shmem, st, P, a, T, m.sc, slot,
                           slot_next, serial, m.partials, fused_args(), Lc, Lg);
        HIP_CHECK(hipGetLastError());
        m.lns_pend = Lc;
        lns_ghost_pending = lns_last_valid = true;   // unpacked by the next fused step or p2p_complete
        if (lns_ghost_prologue) (void)lc_device(Lc);   // (uploaded now, outside any capture, when eager)
        ghost_stale = true;   // lean representation in the ghosts
        lns_fx_steps++;
      } else if (lns_split) {
        if (!m.comm_stream) {
          HIP_CHECK(hipStreamCreateWithFlags(&m.comm_stream, hipStreamNonBlocking));
          HIP_CHECK(hipEventCreateWithFlags(&m.ev_edge, hipEventDisableTiming));
          HIP_CHECK(hipEventCreateWithFlags(&m.ev_halo, hipEventDisableTiming));
        }
        hipLaunchKernelGGL(lk, dim3(lparts ? (1 + T.ne) * T.nbj : ntile), dim3(BLOCK), shmem, st, P, a, T, m.sc, slot,
                           slot_next, serial, m.partials, lparts ? 1 : 0);
      } else {
        hipLaunchKernelGGL(lk, dim3(ntile), dim3(BLOCK), shmem, st, P, a, T, m.sc, slot, slot_next, serial,
                           m.partials, 0);
      }
      HIP_CHECK(hipGetLastError());
      nres = (unsigned)ntile;
      sbuf = 1 - sbuf;
      pbuf = 1 - pbuf;
      cbuf = 1 - cbuf;
      dsbuf = 1 - dsbuf;
      lns_steps++;
      if (lns_split) {
        HIP_CHECK(hipEventRecord(m.ev_edge, st));
        // interior tiles in flight before the exchange is issued; they write
        // neither the edge columns nor the ghost columns
        if (lparts)
          hipLaunchKernelGGL(lk, dim3((T.nbi - 1 - T.ne) * T.nbj), dim3(BLOCK), shmem, st, P, a, T, m.sc, slot,
                             slot_next, serial, m.partials, 2);
        HIP_CHECK(hipGetLastError());
        if (m.local) {   // in-process group: the host orders the streams (see the inviscid path)
          HIP_CHECK(hipEventSynchronize(m.ev_edge));
          exchange(CpuSolver::HALO_LNS, -1, (void*)m.comm_stream);
          HIP_CHECK(hipStreamSynchronize(m.comm_stream));
        } else {
          HIP_CHECK(hipStreamWaitEvent(m.comm_stream, m.ev_edge, 0));
          exchange(CpuSolver::HALO_LNS, -1, (void*)m.comm_stream);
          HIP_CHECK(hipEventRecord(m.ev_halo, m.comm_stream));
          HIP_CHECK(hipStreamWaitEvent(st, m.ev_halo, 0));
        }
        exchange_dt(slot_next);
        overlap_steps++;
      }
    }
  } else {
    if (lean_state) lean_materialize();
    if (lns_state) lns_materialize();
    step_split(P, want_res, slot, slot_next, serial, nblk, false);
  }
  // new-state halo + global dt (MIN over ranks into the next slot)
  if (fx_step) {
    fx_pending = true;   // exchanged inside the tile kernel
  } else if (lns_fx) {
    lns_fx = false;   // exchanged inside the lean N-S kernel + unpacked
  } else if (lnm_split) {
    lnm_split = false;   // exchanged above, overlapped with the interior tiles
  } else if (lns_split) {
    lns_split = false;   // exchanged above, overlapped with the interior tiles
  } else if ((m.comm || m.local || m.p2p.on) && m.nranks > 1) {
    exchange(lns_state ? CpuSolver::HALO_LNS : lean_state ? CpuSolver::HALO_LEAN : CpuSolver::HALO_STATE, slot_next);
  }
  if (!cs.cfg.isAdiabaticWall) {
    SoA s = m.view(h, sbuf, abuf, dsbuf, pbuf);
    hipLaunchKernelGGL(hf2d_wall_solid, dim3(nblk), dim3(BLOCK), 0, st, P, s, m.qdir, c0, c1);
    exchange(CpuSolver::HALO_QDIR);
    hipLaunchKernelGGL(hf2d_wall_wall, dim3(nblk), dim3(BLOCK), 0, st, P, s, m.qdir, c0, c1, m.sc, slot);
    HIP_CHECK(hipGetLastError());
  }
  nstep++;
  lns_prev_mu_t = P.fpa.is_mu_t;
  StepResult r;
  r.async = true;
  if (want_res) {
    hipLaunchKernelGGL(hf2d_reduce_residual, dim3(1), dim3(BLOCK), 0, st, m.partials,
                       (long)nres * nres_waves, m.res_out);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(m.res_host, m.res_out, sizeof(ResidualPack), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    r.res = *m.res_host;
    r.have_residual = true;
  }
  return r;
}

void DeviceSolver::launch_chem(const StepParams& P, const SoA& mid, const SoA& out, long k0, long k1, unsigned nb,
                               int slot) {
  Impl& m = *impl;
#ifdef HF2D_FP32
  (void)P, (void)mid, (void)out, (void)k0, (void)k1, (void)nb, (void)slot, (void)m;
  throw std::runtime_error("FP32 build: finite-rate kinetics need the FP64 build");
#else
  const real* Tprev = m.Tg[pbuf];
  const MechData& md = *cs.cfg.mech->data_ptr();
  const int kind = chem_kernel ? chem_kernel : ((chem_fast && chem_fast_ok) ? 1 : (chem_rtc && chem_rtc_ok) ? 4 : 2);
  if (kind == 4) {
    if (!chem_rtc_ok) throw std::runtime_error("chem_kernel=4: hiprtc kernels unavailable: " + chem_rtc_why);
    if (chem_compact && !m.chem_list) {
      m.chem_list = m.mem.alloc<int>(h.N);
      m.chem_count = m.mem.alloc<unsigned>(1);
    }
    if (!chem_rtc_launch(md, mid, out, Tprev, k0, k1, m.sc, slot, md.Tchem, md.nsub, m.stream,
                         chem_compact ? m.chem_list : nullptr, chem_compact ? m.chem_count : nullptr))
      throw std::runtime_error("hf2d_rtc_chem launch failed");
    chem_kernel_used = "hf2d_rtc_chem";
    return;
  }
  // compiled mechanism: register-resident VALU kernel (chem_fast.hip)
  if (kind == 1) {
    if (!chem_fast_ok) throw std::runtime_error("chem_kernel=1: no compiled kernel for mechanism " + cs.cfg.mech->name);
    if (chem_compact && !m.chem_list) {
      m.chem_list = m.mem.alloc<int>(h.N);
      m.chem_count = m.mem.alloc<unsigned>(1);
    }
    if (!chem_fast_launch(cs.cfg.mech->name, P, mid, out, Tprev, k0, k1, m.sc, slot, md.Tchem, md.nsub, m.stream,
                          chem_compact ? m.chem_list : nullptr, chem_compact ? m.chem_count : nullptr))
      throw std::runtime_error("hf2d_chem_fast launch failed");
    chem_kernel_used = "hf2d_chem_fast";
    return;
  }
  // runtime mechanism: reaction-space algebra on the matrix cores (chem_mech.hip).
  // The dt of the step lives on the device: the kernel takes it from the slot.
  if (kind == 2) {
    if (!m.chem_pack) m.chem_pack = chem_mech_pack(md);
    MechCells q;
    q.S = mid.S;
    q.Yin = mid.Ys;
    q.Yout = out.Ys;
    q.Tprev = Tprev;
    q.Tout = nullptr;
    q.CT = mid.CT;
    q.N = h.N;
    q.c0 = k0;
    q.c1 = k1;
    q.Tchem = md.Tchem;
    q.dt_bits = &m.sc->dt_bits[slot];
    HIP_CHECK((hipError_t)chem_mech_launch(m.chem_pack->dev, q, 0.0, md.nsub, m.stream));
    chem_kernel_used = "hf2d_chem_mech";
    return;
  }
  chem_kernel_used = "hf2d_chem_generic";
  if (m.nsp <= 9)
    hipLaunchKernelGGL(hf2d_chem_generic<9>, dim3(nb), dim3(BLOCK), 0, m.stream, P, mid, out, Tprev, k0, k1, m.sc,
                       slot);
  else
    hipLaunchKernelGGL(hf2d_chem_generic<MECH_MAXSP>, dim3(nb), dim3(BLOCK), 0, m.stream, P, mid, out, Tprev, k0, k1,
                       m.sc, slot);
  HIP_CHECK(hipGetLastError());
#endif
}

void DeviceSolver::synchronize() {
  flush_pending();
  HIP_CHECK(hipStreamSynchronize(impl->stream));
}

// ThreadBlockSize = 0 ("auto-calibrate", UG p.20): time the lean tile
// kernel's geometry choices (cells per thread, tile height) on this device
// and strip, keep the fastest.  Every candidate computes the same bits; the
// state (device arrays and host bookkeeping) is restored afterwards, so the
// run is unaffected apart from its speed.  Only before the first step.
// One traced lean tile step (after `steps` untraced ones): per workgroup the
// phase clocks of lean_tile_body<TR> (TILE_TRACE_WORDS words each, tile order).
std::vector<unsigned long long> DeviceSolver::trace_tile(int steps) {
  if (!lean_ok || cs.cfg.ProblemType == SM_NS || !lean_tile) throw std::runtime_error("trace_tile: lean tile steps only");
  flush_pending();
  const bool g = use_graph;
  use_graph = false;
  if (steps > 0) run_steps(steps);
  const int cpt = lean_cpt == 2 ? 2 : 1;
  const LeanTile T = lean_tile_geom(gi1 - gi0, h.ny, tile_nt(lean_nt, lean_sg && lean_sg_ok), lean_tj, cpt);
  const long n = (long)T.nbi * T.nbj * TILE_TRACE_WORDS * 2;   // room for either cpt
  tile_trace = impl->mem.alloc<unsigned long long>(n);
  try {
    run_steps(2);   // the last step of run_steps stores the output fields (not traced)
    synchronize();
  } catch (...) {
    tile_trace = nullptr;
    use_graph = g;
    throw;
  }
  std::vector<unsigned long long> out(n);
  HIP_CHECK(hipMemcpy(out.data(), tile_trace, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  tile_trace = nullptr;
  use_graph = g;
  while (!out.empty() && out.back() == 0) out.pop_back();
  out.resize((out.size() + TILE_TRACE_WORDS - 1) / TILE_TRACE_WORDS * TILE_TRACE_WORDS);
  return out;
}

std::string DeviceSolver::autotune(int steps) {
  // inviscid lean tile: cells per thread x tile height; lean N-S tile (one
  // cell per thread): tile height (resonator 2000x200: 92 us at the
  // heuristic height, 87 us at 16 rows)
  const bool ns = cs.cfg.ProblemType == SM_NS;
  if (nstep != 0 || iter != 0) return "";
  // mechanism mode: the lean mechanism tile's width (16 x 16: the ring is a
  // second fill on one wavefront; 12 x 16: one fill per thread)
  const bool mech = ns && lean_mech && lnm_ok && cs.cfg.mech_mode();
  if (ns ? !((lean_ns && lns_ok) || mech) : !(lean_ok && lean_tile)) return "";
  flush_pending();
  const real s_dt = dt, s_dtr = dt_running, s_cur = cur_time_part, s_gt = cs.global_time, s_lag = dt_lag;
  const long s_iter = iter, s_last = last_iter;
  const int s_cycle = cycle;
  const bool s_src = isSrcAdd, s_out = step_outputs;
  const ResidualSummary s_res = last_res;
  const bool s_resv = last_res_valid;
  struct Cand {
    int cpt, tj, nt, wgcu = 0;
  };
  std::vector<Cand> cands;
  for (int cpt : {2, 1}) {
    if (ns && cpt == 2) continue;
    if (mech) break;
    for (int tj : {0, 10, 12, 14, 16, 20, 25, 32, 40, 50, 64})
      if ((tj == 0 || tj <= h.ny) && (ns ? tj <= 40 : (tj == 0 || tj >= 16))) cands.push_back({cpt, tj, BLOCK});
  }
  if (mech)   // (Cand::tj carries the tile width here)
    for (int ti : {LNM_TILE, 12}) cands.push_back({1, ti, BLOCK});
  // small workgroups (single-gas inviscid): the geometries of the narrow
  // strips of a multi-GPU run, where 256-thread tiles leave CUs idle
  if (!ns && lean_sg && lean_sg_ok)
    for (int nt : {128, 64})
      for (int cpt : {1, 2})
        for (int tj : {0, 8, 16, 32, 64})
          if (tj <= nt && (tj == 0 || tj <= h.ny)) cands.push_back({cpt, tj, nt});
  double best = 1e30;
  Cand win = mech ? Cand{1, lnm_ti, BLOCK} : Cand{lean_cpt, lean_tj, lean_nt, lean_wgcu};
  char b[160];
  std::string log;
  // same work per candidate whatever the grid (~50 M cell-steps): big grids get fewer steps
  const long cells = std::max(1L, (long)(gi1 - gi0) * h.ny);
  steps = (int)std::max(12L, std::min((long)steps, 50000000L / cells));
  // second stage (inviscid): resident workgroups per CU for the winning
  // geometry (through the LDS request).  Fewer resident workgroups than
  // tiles make later dispatch rounds stage their tiles while earlier ones
  // compute instead of every workgroup loading, then computing, at once.
  bool stage2 = ns;
  for (size_t ci = 0; ci < cands.size(); ci++) {
    const Cand c = cands[ci];
    if (mech) {
      lnm_ti = c.tj;
    } else {
      lean_cpt = c.cpt;
      lean_tj = c.tj;
      lean_nt = c.nt;
      lean_wgcu = c.wgcu;
    }
    graph.reset();   // the state just keeps marching; it is restored once at the end
    double us = 1e30;
    try {
      run_steps(12);   // (first candidate: first lean step) + graph capture
      synchronize();
      for (int rep = 0; rep < 2; rep++) {   // best of two: the candidates differ by a few %
        const auto t0 = std::chrono::steady_clock::now();
        run_steps(steps);
        synchronize();
        us = std::min(us, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / steps * 1e6);
      }
    } catch (const std::exception& e) {   // e.g. the transient went unstable: stop tuning, keep the best so far
      log += std::string("stopped: ") + e.what() + "; ";
      break;
    }
    if (mech)
      std::snprintf(b, sizeof b, "lnm ti=%d %.2f us; ", c.tj, us);
    else if (c.wgcu)
      std::snprintf(b, sizeof b, "wgcu=%d %.2f us; ", c.wgcu, us);
    else if (c.nt == BLOCK)
      std::snprintf(b, sizeof b, "cpt=%d tj=%d %.2f us; ", c.cpt, c.tj, us);
    else
      std::snprintf(b, sizeof b, "nt=%d cpt=%d tj=%d %.2f us; ", c.nt, c.cpt, c.tj, us);
    log += b;
    if (us < best) {
      best = us;
      win = c;
    }
    if (!stage2 && ci + 1 == cands.size()) {
      stage2 = true;
      for (int w : {2, 3, 4, 6, 8, 12, 16}) {
        if (w * (win.nt / WAVE) > 32) break;   // (32 waves per CU)
        Cand c2 = win;
        c2.wgcu = w;
        cands.push_back(c2);
      }
    }
  }
  if (mech) {
    lnm_ti = win.tj;
  } else {
    lean_cpt = win.cpt;
    lean_tj = win.tj;
    lean_nt = win.nt;
    lean_wgcu = win.wgcu;
  }
  // step graphs on or off for the winning geometry: replaying the 6-step
  // graph costs ~1 us per step more than eager launches on the 2000 x 200
  // headline grid (28.5 vs 27.5 us/step over 20-step calls, 1x MI355X,
  // tools/launch_overhead.py) but saves host launch time on small grids
  if (use_graph) {
    double g_us[2] = {1e30, 1e30};
    for (int g : {1, 0}) {
      use_graph = g == 1;
      graph.reset();
      try {
        run_steps(12);
        synchronize();
        for (int rep = 0; rep < 2; rep++) {
          const auto t0 = std::chrono::steady_clock::now();
          run_steps(steps);
          synchronize();
          g_us[g] = std::min(g_us[g],
                             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / steps * 1e6);
        }
      } catch (const std::exception& e) {
        log += std::string("stopped: ") + e.what() + "; ";
        break;
      }
    }
    use_graph = g_us[1] <= g_us[0];
    std::snprintf(b, sizeof b, "graphs on %.2f us, off %.2f us; ", g_us[1], g_us[0]);
    log += b;
  }
  graph.reset();
  dt = s_dt;
  dt_running = s_dtr;
  dt_lag = s_lag;
  cur_time_part = s_cur;
  cs.global_time = s_gt;
  iter = s_iter;
  last_iter = s_last;
  cycle = s_cycle;
  isSrcAdd = s_src;
  step_outputs = s_out;
  last_res = s_res;
  last_res_valid = s_resv;
  upload();   // device scalars from the restored host state
  graph_launches = 0;
  lns_steps = lnm_steps = 0;   // (the tuning steps do not count as the run's)
  if (mech)
    std::snprintf(b, sizeof b, "best lnm ti=%d graphs=%d (%.2f us/step)", win.tj, (int)use_graph, best);
  else
    std::snprintf(b, sizeof b, "best nt=%d cpt=%d tj=%d wgcu=%d graphs=%d (%.2f us/step)", win.nt, win.cpt, win.tj,
                  win.wgcu, (int)use_graph, best);
  return log + b;
}

std::unique_ptr<SolverBase> make_gpu_solver(Case& cs, int device) {
  return std::unique_ptr<SolverBase>(new DeviceSolver(cs, device < 0 ? 0 : device));
}

// Strip rank of the native multi-process CLI (hf2d_main.cpp).  `boot` is the
// host communicator (TCP): it carries the driver's host reductions and the
// p2p bootstrap -- every rank exports its xGMI mailbox descriptor, the
// descriptors are all-gathered and imported, one poisoned full-state exchange
// is checksummed on every rank (p2p_probe), and the ranks agree on the
// result.  If any rank fails (or transport "rccl" is asked for), the RCCL
// unique id travels through `boot` and every rank uses grouped RCCL
// send/recv on the solver stream instead.  `used` reports the transport.
std::unique_ptr<SolverBase> make_gpu_strip_solver(Case& cs, int device, int gi0, int gi1, Comm& boot,
                                                  const std::string& transport, std::string& used) {
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  // more local ranks than GPUs (tests on a one-GPU box): ranks share devices
  if (device >= ndev && ndev > 0) device %= ndev;
  std::unique_ptr<DeviceSolver> s(new DeviceSolver(cs, device < 0 ? 0 : device, gi0, gi1));
  used = "none";
  if (cs.cfg.ThreadBlockSize == 0) {
    const char* at = std::getenv("HF2D_AUTOTUNE");
    if (!at || std::string(at) != "0") s->autotune();
  }
  if (boot.size() == 1) return std::unique_ptr<SolverBase>(s.release());
  const int r = boot.rank(), n = boot.size();
  auto use_rccl = [&] {
    const std::string uid = boot.allgather_bytes(r == 0 ? DeviceSolver::nccl_unique_id() : std::string())[0];
    s->init_comm(uid, r, n);
    used = "rccl";
  };
  if (transport != "p2p") {
    use_rccl();
    return std::unique_ptr<SolverBase>(s.release());
  }
  // host-side reductions of the driver (output steps) over the bootstrap
  // communicator; the halos and the per-step dt MIN go through the mailboxes
  s->comm = &boot;
  std::string desc, why;
  int bad = 0;
  try {
    desc = s->p2p_export(r, n);
  } catch (const std::exception& e) {
    bad = 1;
    why = e.what();
  }
  const std::vector<std::string> descs = boot.allgather_bytes(bad ? std::string() : desc);
  for (const std::string& d : descs) bad |= d.empty() ? 1 : 0;
  if (!bad) {
    try {
      s->p2p_import(descs);
    } catch (const std::exception& e) {
      bad = 1;
      why = e.what();
    }
  }
  if (boot.allreduce_max_int(bad) == 0) {
    // self-validation: one poisoned full-state exchange, checksummed
    const std::vector<std::string> probes = boot.allgather_bytes(s->p2p_probe());
    if (!DeviceSolver::p2p_probe_ok(probes, r, &why)) bad = 1;
  } else {
    bad = 1;
  }
  if (boot.allreduce_max_int(bad) == 0) {
    used = "p2p";
    const char* f = std::getenv("HF2D_P2P_FUSE");
    s->p2p_fuse = !(f && std::string(f) == "0");
  } else {
    use_rccl();
    s->p2p_fallback();
    if (!why.empty()) std::fprintf(stderr, "[hf2d rank %d] p2p transport unavailable (%s); using RCCL\n", r, why.c_str());
  }
  return std::unique_ptr<SolverBase>(s.release());
}

}  // namespace hf2d
