#include "gasdyn.hpp"

#include <cmath>

namespace hf2d {

GasFlow::GasFlow(real Cp, real T0, real P0, real R, real lam_, real mu_) {
  lambda_ = 0.01;
  C = Cp;
  k_ = C / (C - R);
  t0_ = T0;
  p0_ = P0;
  r_ = R;
  C = k_ * r_ / (k_ - 1);
  lam = lam_;
  mu = mu_;
}

GasFlow GasFlow::make2d(real mu, real lam, real Cp, real T, real P, real R, real u, real v) {
  GasFlow f(Cp, T, P, R, lam, mu);
  f.is2d_ = true;
  f.uu_ = u;
  f.vv_ = v;
  f.flow_Wg(std::sqrt(u * u + v * v + 1.e-12));
  return f;
}

GasFlow GasFlow::as2d() const {
  GasFlow f = *this;
  f.is2d_ = true;
  // The reference constructs Flow2D(Flow&) with UU = Wg() evaluated on
  // uninitialised members; we use the 1-D speed along +x instead.
  f.uu_ = flow_Wg();
  f.vv_ = 0;
  return f;
}

real GasFlow::LMAX() const { return std::sqrt((k_ + 1) / (k_ - 1)); }
real GasFlow::Akr() const { return std::sqrt(2 * k_ / (k_ + 1) * r_ * t0_); }
real GasFlow::Asound() const { return std::sqrt(k_ * r_ * t0_ * TAU()); }
real GasFlow::tau_of(real l) const { return (1 - (k_ - 1) / (k_ + 1) * l * l); }
real GasFlow::pf_of(real l) const { return std::pow(tau_of(l), k_ / (k_ - 1)); }
real GasFlow::eps_of(real l) const { return std::pow(tau_of(l), 1 / (k_ - 1)); }
real GasFlow::qf_of(real l) const {
  real r = std::pow((k_ + 1) / 2, 1 / (k_ - 1)) * l;
  return r * std::pow(1 - (k_ - 1) / (k_ + 1) * l * l, 1 / (k_ - 1));
}

real GasFlow::flow_LAM(real l) {
  if (LMAX() > l && l > 0.) {
    lambda_ = l;
    return lambda_;
  }
  return -1;
}

real GasFlow::flow_Wg(real w) {
  if (w > 0.) {
    if (w < Akr() * LMAX())
      lambda_ = w / Akr();
    else
      return -1;
    return w;
  }
  return -1;
}

real GasFlow::flow_MACH(real m) {
  if (m < 0.) return -1;
  lambda_ = std::sqrt((k_ + 1) / 2 * m * m / (1 + ((k_ - 1) / 2 * m * m)));
  return m;
}

// Bisection on tau(lambda) with the reference's 1 % tolerance (flow.cpp:320-362).
real GasFlow::bisect_tau(real val) {
  real lmax = LMAX(), lmin = 0.01, test;
  int iter = 0;
  do {
    iter++;
    test = (lmax + lmin) / 2;
    if (tau_of(test) < val)
      lmax = test;
    else
      lmin = test;
    if (iter > 100) return -1;
  } while (std::fabs((val - tau_of(test)) / val) > 0.01);
  return test;
}

real GasFlow::Tg(real T) {
  if (t0_ > T && T > 0.) {
    lambda_ = bisect_tau(T / t0_);
    return Tg();
  }
  return -1;
}

void GasFlow::CorrectFlow(real T, real p, real ref_val, bool fixed_mach) {
  real res_p, res_t;
  int iter = 0;
  do {
    if (fixed_mach)
      flow_MACH(ref_val);
    else
      flow_MACH(ref_val / Asound());
    t0_ = T / TAU();
    p0_ = p / PF();
    res_p = std::fabs((p0_ - p / PF()) / p0_);
    res_t = std::fabs((t0_ - T / TAU()) / t0_);
    if (fixed_mach)
      flow_Wg(ref_val * Asound());
    else
      flow_Wg(ref_val);
    iter++;
  } while ((res_p > 0.0001 || res_t > 0.0001) && iter < 100);
}

real GasFlow::Wg2d() const { return std::sqrt(uu_ * uu_ + vv_ * vv_ + 1.e-5); }

real GasFlow::MACH2d(real m) {
  if (vv_ != 0.0) {
    real angle = std::atan(vv_ / uu_);
    flow_MACH(m);
    uu_ = flow_Wg() * std::cos(angle);
    vv_ = flow_Wg() * std::sin(angle);
  } else {
    flow_MACH(m);
    if (vv_ == 0.0) {
      uu_ = flow_Wg();
    } else if (uu_ == 0.0) {
      vv_ = flow_Wg();
    }
  }
  return flow_MACH();
}

real GasFlow::set_U(real u) {
  uu_ = u;
  flow_Wg(std::sqrt(uu_ * uu_ + vv_ * vv_ + 1.e-12));
  return uu_;
}
real GasFlow::set_V(real v) {
  vv_ = v;
  flow_Wg(std::sqrt(uu_ * uu_ + vv_ * vv_ + 1.e-12));
  return vv_;
}
real GasFlow::set_UV(real u, real v) {
  uu_ = u;
  vv_ = v;
  return flow_Wg(std::sqrt(uu_ * uu_ + vv_ * vv_ + 1.e-12));
}

}  // namespace hf2d
