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
  unsigned pad2;
};

__device__ inline double bits_to_d(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ inline unsigned long long d_to_bits(double d) { return (unsigned long long)__double_as_longlong(d); }

// Step n reads slot n%3, min-reduces into (n+1)%3 and resets (n+2)%3.
__host__ __device__ inline int slot_reset(int slot) { return (slot + 2) % 3; }

__device__ inline void apply_dt(StepParams& P, const DevScalars* sc, int slot) {
  const double dt = bits_to_d(sc->dt_bits[slot]);
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
