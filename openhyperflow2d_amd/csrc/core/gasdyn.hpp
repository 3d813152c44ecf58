// One-dimensional isentropic gas-dynamics functions in the critical-velocity
// ratio lambda, used to build boundary / initial states from the deck.
// Behavioural reference: libFlow/flow.hpp:20-132, libFlow/flow.cpp:9-406,
// libFlow/flow2d.hpp:13-110, libFlow/flow2d.cpp:10-63.
//
// The reference splits this into Flow and Flow2D with C++ name hiding
// deciding which overload runs; here the 1-D ("flow_*") and 2-D ("*2d")
// operations are separate, explicitly named methods of one class.
#pragma once

#include "common.hpp"

namespace hf2d {

class GasFlow {
 public:
  // Flow(Cp, T0, P0, R, lam, mu)
  GasFlow(real Cp, real T0, real P0, real R, real lam_ = 0.01, real mu_ = 5.e-5);
  // Flow2D(mu, lam, Cp, T, P, R, u, v)
  static GasFlow make2d(real mu, real lam, real Cp, real T, real P, real R, real u, real v);

  // --- 1-D (Flow) interface ---
  real kg() const { return k_; }
  real Rg() const { return r_; }
  real T0() const { return t0_; }
  real P0() const { return p0_; }
  real LAM() const { return lambda_; }
  real LMAX() const;
  real TAU() const { return tau_of(lambda_); }
  real PF() const { return pf_of(lambda_); }
  real EPS() const { return eps_of(lambda_); }
  real QF() const { return qf_of(lambda_); }
  real Tg() const { return t0_ * TAU(); }
  real Pg() const { return p0_ * PF(); }
  real ROG() const { return EPS() * P0() / Rg() / T0(); }
  real Akr() const;
  real Asound() const;
  real flow_Wg() const { return lambda_ * Akr(); }
  real flow_MACH() const { return flow_Wg() / Asound(); }
  real flow_LAM(real l);          // Flow::LAM(new)
  real flow_Wg(real w);           // Flow::Wg(new)
  real flow_MACH(real m);         // Flow::MACH(new)
  real Tg(real T);                // Flow::Tg(new) (bisection)
  void CorrectFlow(real T, real p, real ref_val, bool fixed_mach);

  // --- 2-D (Flow2D) interface ---
  real U() const { return uu_; }
  real V() const { return vv_; }
  real Wg2d() const;                 // sqrt(U^2+V^2+1e-5)
  real MACH2d(real m);               // keeps the flow angle
  real set_U(real u);
  real set_V(real v);
  real set_UV(real u, real v);       // Flow2D::Wg(u, v)
  bool is2d() const { return is2d_; }

  real C = 0, lam = 0, mu = 0;       // Cp, conductivity, viscosity

  // Flow2D(Flow&) conversion used by Area fill with a 1-D flow.
  GasFlow as2d() const;

 private:
  GasFlow() = default;
  real tau_of(real l) const;
  real pf_of(real l) const;
  real eps_of(real l) const;
  real qf_of(real l) const;
  real bisect_tau(real val);
  real r_ = 300, t0_ = 300, p0_ = 1e5, lambda_ = 0.01, k_ = 1.4;
  real uu_ = 0, vv_ = 0;
  bool is2d_ = false;
};

}  // namespace hf2d
