// Residual / time-step reduction pack shared by the CPU steppers, the HIP
// reduction kernels and the multi-rank all-gather.  Mirrors the reference's
// per-rank Var_pack (dt_min + 9 x DD_pack; deeps2d_core.cpp:502-510) but is
// reduced deterministically on every rank instead of being gathered to 0.
#pragma once

#include <cmath>

#include "common.hpp"

namespace hf2d {

struct EqResidual {
  real dd_max;   // max relative residual
  real rms;      // sum DD^2 (standard) or sum dS^2 (alternate)
  real sum_div;  // sum S^2 (alternate)
  real count;    // number of contributing cells
  int i, j;      // argmax location (global indices)
};

struct ResidualPack {
  real dt_min;
  EqResidual eq[NEQ];
};

HF_HD inline void residual_reset(ResidualPack& r) {
  r.dt_min = 1.0;
  for (int k = 0; k < NEQ; k++) {
    r.eq[k].dd_max = 0;
    r.eq[k].rms = 0;
    r.eq[k].sum_div = 0;
    r.eq[k].count = 0;
    r.eq[k].i = 0;
    r.eq[k].j = 0;
  }
}

// Combine b into a (order matters only for argmax ties: a wins).
HF_HD inline void residual_merge(ResidualPack& a, const ResidualPack& b) {
  a.dt_min = a.dt_min < b.dt_min ? a.dt_min : b.dt_min;
  for (int k = 0; k < NEQ; k++) {
    if (b.eq[k].dd_max > a.eq[k].dd_max) {
      a.eq[k].dd_max = b.eq[k].dd_max;
      a.eq[k].i = b.eq[k].i;
      a.eq[k].j = b.eq[k].j;
    }
    a.eq[k].rms += b.eq[k].rms;
    a.eq[k].sum_div += b.eq[k].sum_div;
    a.eq[k].count += b.eq[k].count;
  }
}

// Deterministic, associative merge used by tree reductions: the argmax keeps
// the larger residual and, on ties, the cell that comes later in the
// reference's sweep order (x outer, y inner), matching its "last equal wins".
HF_HD inline void residual_merge_lex(ResidualPack& a, const ResidualPack& b) {
  a.dt_min = a.dt_min < b.dt_min ? a.dt_min : b.dt_min;
  for (int k = 0; k < NEQ; k++) {
    const EqResidual& e = b.eq[k];
    EqResidual& f = a.eq[k];
    const bool later = (e.i > f.i) || (e.i == f.i && e.j > f.j);
    if (e.dd_max > f.dd_max || (e.dd_max == f.dd_max && later)) {
      f.dd_max = e.dd_max;
      f.i = e.i;
      f.j = e.j;
    }
    f.rms += e.rms;
    f.sum_div += e.sum_div;
    f.count += e.count;
  }
}

// Final RMS per equation (MPI definition, deeps2d_core.cpp:1506-1518) and the
// maximum used by the exit monitor.
struct ResidualSummary {
  real rms[NEQ];
  real max_rms;
  int k_max;
};

inline ResidualSummary residual_finalize(const ResidualPack& p, int alternate, int monitor_index,
                                         bool serial = false, real exit_value = 0) {
  ResidualSummary s;
  s.max_rms = (serial && monitor_index < 5) ? 0.5 * exit_value : 0;
  s.k_max = -1;
  for (int k = 0; k < NEQ; k++) {
    real r = p.eq[k].rms;
    if (alternate) {
      if (r > 0.0 && p.eq[k].sum_div > 0)
        r = std::sqrt(r / p.eq[k].sum_div);
      else if (serial)
        r = 0.0;   // serial build: sqrt only of positive sums, else 0
    } else {
      if (p.eq[k].count > 0 && (!serial || r > 0.0))
        r = std::sqrt(r / p.eq[k].count);
      else if (serial)
        r = 0.0;
    }
    s.rms[k] = r;
  }
  for (int k = 0; k < NEQ; k++) {
    if (monitor_index == 0 || monitor_index > 4) {
      if (s.rms[k] >= s.max_rms) {
        s.max_rms = s.rms[k];
        s.k_max = k;
      }
    } else {
      if (s.rms[monitor_index - 1] >= s.max_rms) {
        s.max_rms = s.rms[monitor_index - 1];
        s.k_max = monitor_index - 1;
      }
    }
  }
  return s;
}

}  // namespace hf2d
