// Device-side helpers shared by the HIP translation units of the solver.
#pragma once

#include <hip/hip_runtime.h>

#include "../core/stepkern.hpp"

namespace hf2d {

// Per-step scalars living on the device.
struct DevScalars {
  unsigned long long dt_bits[3];   // rotating dt slots (IEEE bits of positive doubles)
  double iter[3];                  // iteration number of the step using the slot
  double beta_min[3], cfl_min[3];  // scenario values of that iteration
  double time_part;                // accumulated dt since the cycle start
  int neg_T;
  int pad;
  double dt_val[3];                // dt of the step that used the slot (the lean
                                   // mechanism step's fill belongs to the previous one)
  unsigned hot_cnt[3];             // lean mechanism step: reacting cells listed by the step using the slot
  unsigned hot_cnt2[3];            // ... by its interior tiles (comm-overlap steps: a second list)
  // Lagged dt (StepParams::lag_dt): dt_lag[slot] is the dt of the step that
  // reads the slot -- the all-rank MIN of two steps back.  The first kernel
  // of step n (lag_head) moves MIN(slot n) -- the previous step's MIN, folded
  // over the ranks -- to dt_lag[slot of n + 1] before it overwrites the word.
  unsigned long long dt_lag[3];
  // Sharded dt MIN: every workgroup of a step used to atomicMin into ONE word,
  // and device-scope atomics to one address serialise at the memory side
  // (~10 ns each: the 800 workgroups of a small-strip step queued ~7 us
  // behind them).  Workgroup b min-reduces into shard
  // b % DT_SHARDS (one 128-byte line each) instead; the value of a slot is
  // MIN(dt_bits[slot], its shards) (dt_get), and folds that publish a
  // global MIN store it into dt_bits[slot] (the shards stay >= it).
  alignas(128) unsigned long long dt_sh[3][16][16];
};
constexpr int DT_SHARDS = 16;

__device__ inline double bits_to_d(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ inline unsigned long long d_to_bits(double d) { return (unsigned long long)__double_as_longlong(d); }

// Step n reads slot n%3, min-reduces into (n+1)%3 and resets (n+2)%3.
__host__ __device__ inline int slot_reset(int slot) { return (slot + 2) % 3; }

// (IEEE bits of positive doubles order like the values)
__host__ __device__ inline unsigned long long dt_bits_min(unsigned long long a, unsigned long long b) {
  return a < b ? a : b;
}
// value of a dt slot: the word and its shards (plain loads: the producers
// are earlier kernels)
__device__ inline double dt_get(const DevScalars* sc, int slot) {
  unsigned long long b = sc->dt_bits[slot];
#pragma unroll
  for (int k = 0; k < DT_SHARDS; k++) b = dt_bits_min(b, sc->dt_sh[slot][k][0]);
  return bits_to_d(b);
}
// same inside the producing kernel, after its workgroups' atomics (relaxed
// agent-scope loads)
__device__ inline double dt_get_fresh(DevScalars* sc, int slot) {
  unsigned long long b = __hip_atomic_load(&sc->dt_bits[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < DT_SHARDS; k++)
    b = dt_bits_min(b, __hip_atomic_load(&sc->dt_sh[slot][k][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return bits_to_d(b);
}
// a step's contribution (one thread per workgroup)
__device__ inline void dt_min(DevScalars* sc, int slot, double m) {
  atomicMin(&sc->dt_sh[slot][blockIdx.x % DT_SHARDS][0], d_to_bits(m));
}
__device__ inline void dt_reset(DevScalars* sc, int slot) {
  const unsigned long long one = d_to_bits(1.0);
  sc->dt_bits[slot] = one;
#pragma unroll
  for (int k = 0; k < DT_SHARDS; k++) sc->dt_sh[slot][k][0] = one;
}
__host__ inline unsigned long long dt_get_host(const DevScalars& s, int slot) {
  unsigned long long b = s.dt_bits[slot];
  for (int k = 0; k < DT_SHARDS; k++) b = dt_bits_min(b, s.dt_sh[slot][k][0]);
  return b;
}
__host__ inline void dt_set_host(DevScalars& s, int slot, unsigned long long b) {
  s.dt_bits[slot] = b;
  for (int k = 0; k < DT_SHARDS; k++) s.dt_sh[slot][k][0] = b;
}

// dt_get with one vector load per lane (lane k < DT_SHARDS: shard k, lane
// DT_SHARDS: the word) and a cross-lane MIN: the loads wait on vmcnt with the
// tile staging instead of on lgkmcnt with its LDS stores.  Every lane of the
// wavefront must be active.
__device__ inline double dt_get_wave(const DevScalars* sc, int slot) {
  const int lane = (int)(threadIdx.x & 63);
  unsigned long long b = ~0ull;
  if (lane < DT_SHARDS) b = sc->dt_sh[slot][lane][0];
  else if (lane == DT_SHARDS) b = sc->dt_bits[slot];
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) b = dt_bits_min(b, (unsigned long long)__shfl_xor((long long)b, off, 64));
  return bits_to_d((unsigned long long)__shfl((long long)b, 0, 64));
}

// dt of the step reading the slot
__device__ inline double dt_cur(const StepParams& P, const DevScalars* sc, int slot) {
  return __builtin_expect(P.lag_dt != 0, 0) ? bits_to_d(sc->dt_lag[slot]) : dt_get(sc, slot);
}
// the lean tile kernel's read (StepParams::dt_read)
__device__ inline double dt_cur_tile(const StepParams& P, const DevScalars* sc, int slot) {
  if (__builtin_expect(P.lag_dt != 0, 0)) return bits_to_d(sc->dt_lag[slot]);
  if (P.dt_read == 2) return bits_to_d(sc->dt_bits[slot]);
  if (P.dt_read == 1) return dt_get_wave(sc, slot);
  return dt_get(sc, slot);
}
// first kernel of a lagged step, one thread, before the slot's word is
// overwritten with this step's dt: the previous step's MIN goes to the next
// step's lag word (fold: the MIN over the other ranks, if it is still pending)
__device__ inline void lag_head(const StepParams& P, DevScalars* sc, int slot, int slot_next, double fold = 1.0) {
  if (P.lag_dt) {
    const double m = dt_get(sc, slot);
    sc->dt_lag[slot_next] = d_to_bits(fold < m ? fold : m);
  }
}

__device__ inline void apply_dt(StepParams& P, const DevScalars* sc, int slot, bool tile = false) {
  const double dt = tile ? dt_cur_tile(P, sc, slot) : dt_cur(P, sc, slot);
  P.dt = dt;
  P.dtdx = dt / P.dx;
  P.dtdy = dt / P.dy;
  if (P.scen) {   // scenario values of this step's iteration (scenario_next)
    P.beta_min = sc->beta_min[slot];
    P.CFL_min = sc->cfl_min[slot];
  }
}

// Run once per step by one thread of the step's first kernel: iteration
// number and CFL / beta scenario values (SolverBase::make_params arithmetic)
// of the next step.
__device__ inline void scenario_next(const StepParams& P, DevScalars* sc, int slot, int slot_next) {
  const double it = sc->iter[slot] + 1.0;
  sc->iter[slot_next] = it;
  if (P.scen) {
    const real bs = table_eval(P.scen->beta, it), cs = table_eval(P.scen->cfl, it);
    sc->beta_min[slot_next] = (bs < P.scen->beta0) ? bs : P.scen->beta0;   // std::min(beta0, bs)
    sc->cfl_min[slot_next] = (cs < P.scen->CFL) ? cs : P.scen->CFL;
  }
}

}  // namespace hf2d
