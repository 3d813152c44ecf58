#include "postproc.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <vector>

namespace hf2d {

std::string plt_header(const Case& cs, real global_time, int ncols) {
  const Config& C = cs.cfg;
  char h1[1024], h2[256];
  std::snprintf(h1, sizeof h1,
                "VARIABLES = X, %s, U, V, T, p, Rho, Y_fuel, Y_ox, Y_cp, Y_i, %s, Mach, l_min, y+, Cp\n",
                C.FT == 1 ? "R" : "Y", C.is_p_asterisk_out ? "p*" : "mu_t/mu");
  std::snprintf(h2, sizeof h2, "ZONE T=\"Time: %g sec.\" I= %i J= %i F=POINT\n", global_time, ncols, C.MaxY);
  return std::string(h1) + h2;
}

const GasFlow* plt_cx_flow(const Case& cs) {
  const Config& C = cs.cfg;
  return (C.is_Cx_calc && C.Cx_Flow_index >= 1 && C.Cx_Flow_index <= (int)cs.flows2d.size())
             ? &cs.flows2d[C.Cx_Flow_index - 1]
             : nullptr;
}

void plt_row(std::ostream& o, const Case& cs, const Field& J, int j, int ib, int ie, const GasFlow* cxf) {
  const Config& C = cs.cfg;
  const real dx_out = (C.dx * C.MaxX) / (C.MaxX - 1);
  const real dy_out = (C.dy * C.MaxY) / (C.MaxY - 1);
  for (int i = ib; i < ie; i++) {
    const CellRecord& n = J.at(i, j);
    o << i * dx_out * 1.e3 << "  ";
    o << dy_out * j * 1.e3 << "  ";
    real Mach = 0;
    if (!n.is(CT_SOLID)) {
      o << n.U << "  " << n.V << "  " << n.Tg << "  " << n.p << "  " << n.S[0] << "  ";
      const real A = std::sqrt(n.k * n.R * n.Tg + 1.e-30);
      const real W = std::sqrt(n.U * n.U + n.V * n.V + 1.e-30);
      Mach = W / A;
      if (n.S[0] != 0.) {
        o << n.S[4] / n.S[0] << "  " << n.S[5] / n.S[0] << "  " << n.S[6] / n.S[0] << "  ";
        o << std::fabs(1 - n.S[4] / n.S[0] - n.S[5] / n.S[0] - n.S[6] / n.S[0]) << "  ";
        if (C.is_p_asterisk_out)
          o << p_asterisk(n) << "  ";
        else
          o << n.mu_t / n.mu << "  ";
      } else {
        o << " +0. +0  +0  +0  +0  ";
      }
    } else {
      o << "  0  0  " << n.Tg << "  0  0  0  0  0  0  0";
    }
    if (!n.is(CT_SOLID)) {
      if (Mach > 1.e-30)
        o << Mach << "  " << n.l_min << " " << n.y_plus;
      else
        o << "  0  0  0  ";
    } else {
      o << "  0  0  0  ";
    }
    if (C.is_Cx_calc && cxf)
      o << " " << calc_cp(n, *cxf) << "\n";
    else
      o << " 0\n";
  }
}

void save_field_plt(const std::string& path, const Case& cs, const Field& J, real global_time, bool rewrite) {
  save_field_plt_cols(path, cs, J, global_time, rewrite, 0, cs.cfg.MaxX);
}

void save_field_plt_cols(const std::string& path, const Case& cs, const Field& J, real global_time, bool rewrite,
                         int ib, int ie) {
  if (!J.resident(ib) || !J.resident(ie - 1)) throw std::runtime_error("save_field_plt: columns not resident");
  std::ofstream o(path, rewrite ? std::ios::trunc : std::ios::app);
  o << plt_header(cs, global_time, ie - ib);
  const GasFlow* cxf = plt_cx_flow(cs);
  for (int j = 0; j < cs.cfg.MaxY; j++) {
    plt_row(o, cs, J, j, ib, ie, cxf);
    if (rewrite) o << "\n";
  }
}

void save_rms_header(const std::string& path, const Config& C) {
  std::ofstream o(path, std::ios::trunc);
  o << "#VARIABLES = N, RMS_Ro(N), RMS_RoU(N), RMS_RoV(N), RMS_RoE(N), RMS_RoY_fu(N), RMS_RoY_ox(N), "
       "RMS_RoY_cp(N), RMS_k(N), RMS_eps(N)"
    << (C.is_Cd_calc ? ", Cd(N), Cv(N)" : "") << "\n";
}

void append_rms(const std::string& path, long n, const real* rms, const Config& C, const real* cd_cv) {
  std::ofstream o(path, std::ios::app);
  o << n << " ";
  for (int i = 0; i < NEQ; i++) o << rms[i] << " ";
  if (cd_cv) o << " " << cd_cv[0] << " " << cd_cv[1] << " ";
  o << "\n";
}

void save_monitors_header(const std::string& path, const Config& C) {
  std::ofstream o(path, std::ios::trunc);
  o << "#VARIABLES = Time";
  for (size_t i = 0; i < C.monitors.size(); i++) o << ", Point-" << i + 1 << ".p, Point-" << i + 1 << ".T";
  o << "\n";
}

void append_monitors(const std::string& path, real t, const std::vector<MonitorPoint>& m) {
  std::ofstream o(path, std::ios::app);
  o << t << " ";
  for (auto& p : m) o << p.p << " " << p.T << " ";
  o << "\n";
}

real p_asterisk(const CellRecord& n) {
  const real A = std::sqrt(n.k * n.R * n.Tg);
  const real WW = std::sqrt(n.U * n.U + n.V * n.V);
  const real Mach = WW / A;
  return n.p * std::pow(1.0 + (n.k - 1.0) * 0.5 * Mach * Mach, n.k / (n.k - 1.0));
}
real T_asterisk(const CellRecord& n) { return n.CP > 0. ? (n.U * n.U + n.V * n.V) * 0.5 / n.CP : 0.; }
real schlieren(const CellRecord& n) { return std::sqrt(n.dSdx[0] * n.dSdx[0] + n.dSdy[0] * n.dSdy[0]); }
real re_airfoil(real chord, const GasFlow& f) { return f.Wg2d() * chord * f.ROG() / f.mu; }

real calc_area(const Case& cs, const Field& J, real x0, real y0, real dy) {
  const Config& C = cs.cfg;
  const unsigned i = (unsigned)(x0 / C.dx);
  const unsigned j0 = (unsigned)(y0 / C.dy), j1 = (unsigned)((y0 + dy) / C.dy);
  real Sp = 0;
  if ((int)i >= J.nx) return 0;
  for (int j = (int)j0; j < (int)j1 && j < J.ny; j++) {
    const CellRecord& n = J.at(i, j);
    if (!n.is(CT_SOLID)) Sp += (C.FT == FT_FLAT) ? C.dy : 2 * M_PI * C.dy * n.y;
  }
  return Sp;
}

real mass_flow_rate_x(const Case& cs, const Field& J, real x0, real y0, real dy) {
  const Config& C = cs.cfg;
  const unsigned i = (unsigned)(x0 / C.dx);
  const unsigned j0 = (unsigned)(y0 / C.dy), j1 = (unsigned)((y0 + dy) / C.dy);
  real Mp = 0;
  if ((int)i >= J.nx) return 0;
  for (int j = (int)j0; j < (int)j1 && j < J.ny; j++) {
    const CellRecord& n = J.at(i, j);
    if (!n.is(CT_SOLID)) Mp += (C.FT == FT_FLAT) ? C.dy * n.S[I_RHOU] : 2 * M_PI * C.dy * n.y * n.S[I_RHOU];
  }
  return Mp;
}

static bool in_box(const Config& C, int i, int j, real x0, real y0, real dx, real dy) {
  return i >= (int)(x0 / C.dx) && i <= (int)((x0 + dx) / C.dx) && j >= (int)(y0 / C.dy) && j <= (int)((y0 + dy) / C.dy);
}

void x_force_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                   std::vector<real>& fp, std::vector<real>& fd) {
  const Config& C = cs.cfg;
  for (int i = ib; i < ie; i++)
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& n = J.at(i, j);
      if (!((n.is(CT_WALL_LAW) || n.is(CT_WALL_NO_SLIP)) && in_box(C, i, j, x0, y0, dx, dy))) continue;
      real Sp, Sd;
      if (C.FT == FT_FLAT) {
        Sp = C.dy;
        Sd = C.dx;
      } else {
        Sp = 2 * M_PI * (j + 0.5) * C.dy * C.dy;
        Sd = 2 * M_PI * (j + 0.5) * C.dy * C.dx;
      }
      // Fp -= x is Fp += -x exactly: the terms are folded in this order
      if (i > 0 && J.at(i - 1, j).is(CT_SOLID))
        fp.push_back(-(Sp * n.p));
      else if (i < J.nx - 1 && J.at(i + 1, j).is(CT_SOLID))
        fp.push_back(Sp * n.p);
      const real tau = Sd * (n.mu + n.mu_t) * std::fabs(n.dUdy);
      if (j < J.ny - 1 && !J.at(i, j + 1).is(CT_SOLID)) {
        fd.push_back(J.at(i, j + 1).U > 0 ? tau : -tau);
      } else if (j > 0 && !J.at(i, j - 1).is(CT_SOLID)) {
        fd.push_back(J.at(i, j - 1).U > 0 ? tau : -tau);
      }
    }
}

void y_force_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                   std::vector<real>& fp, std::vector<real>& fd) {
  const Config& C = cs.cfg;
  for (int i = ib; i < ie; i++)
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& n = J.at(i, j);
      if (!((n.is(CT_WALL_LAW) || n.is(CT_WALL_NO_SLIP)) && in_box(C, i, j, x0, y0, dx, dy))) continue;
      real Sp, Sd;
      if (C.FT == FT_FLAT) {
        Sp = C.dx;
        Sd = C.dy;
      } else {
        Sp = 2 * M_PI * n.y * C.dx;
        Sd = 2 * M_PI * n.y * C.dy;
      }
      if (j > 0 && J.at(i, j - 1).is(CT_SOLID))
        fp.push_back(-(Sp * n.p));
      else if (j < J.ny - 1 && J.at(i, j + 1).is(CT_SOLID))
        fp.push_back(Sp * n.p);
      const real tau = -Sd * (n.mu + n.mu_t) * std::fabs(n.dVdx);
      if (i < J.nx - 1 && !J.at(i + 1, j).is(CT_SOLID)) {
        fd.push_back(J.at(i + 1, j).V > 0 ? tau : -tau);
      } else if (i > 0 && !J.at(i - 1, j).is(CT_SOLID)) {
        fd.push_back(J.at(i - 1, j).V > 0 ? tau : -tau);
      }
    }
}

real fold_terms(const std::vector<real>& t) {
  real s = 0;
  for (real v : t) s += v;
  return s;
}

real x_force(const Case& cs, const Field& J, real x0, real y0, real dx, real dy) {
  std::vector<real> fp, fd;
  x_force_terms(cs, J, x0, y0, dx, dy, 0, J.nx, fp, fd);
  return fold_terms(fp) + fold_terms(fd);
}

real y_force(const Case& cs, const Field& J, real x0, real y0, real dx, real dy) {
  std::vector<real> fp, fd;
  y_force_terms(cs, J, x0, y0, dx, dy, 0, J.nx, fp, fd);
  return fold_terms(fp) + fold_terms(fd);
}

// CalcXForceYSym2D (out_cfd_param.cpp:199-254): x force on the wall cells of
// x in [x0, x0+l], j <= d/dy; axisymmetric areas use the cell's y (not j+0.5).
real x_force_ysym(const Case& cs, const Field& J, real x0, real l, real d) {
  const Config& C = cs.cfg;
  real Fp = 0, Fd = 0;
  const int i0 = (int)(x0 / C.dx), i1 = (int)((l + x0) / C.dx), j1 = (int)(d / C.dy);
  for (int i = 0; i < J.nx; i++)
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& n = J.at(i, j);
      if (!((n.is(CT_WALL_LAW) || n.is(CT_WALL_NO_SLIP)) && i >= i0 && i <= i1 && j <= j1)) continue;
      const real Sp = (C.FT == FT_FLAT) ? C.dy : 2 * M_PI * n.y * C.dy;
      const real Sd = (C.FT == FT_FLAT) ? C.dx : 2 * M_PI * n.y * C.dx;
      if (i > 0 && J.at(i - 1, j).is(CT_SOLID))
        Fp -= Sp * n.p;
      else if (i < J.nx - 1 && J.at(i + 1, j).is(CT_SOLID))
        Fp += Sp * n.p;
      const real tau = -Sd * (n.mu + n.mu_t) * std::fabs(n.dUdy);
      if (j < J.ny - 1 && !J.at(i, j + 1).is(CT_SOLID))
        Fd += J.at(i, j + 1).U > 0 ? tau : -tau;
      else if (j > 0 && !J.at(i, j - 1).is(CT_SOLID))
        Fd += J.at(i, j - 1).U > 0 ? tau : -tau;
    }
  return Fp + Fd;
}

// GetFmid (out_cfd_param.cpp:391-429): frontal (mid-section) area of the wall
// rows inside the box -- dy per row (flat) or the 2*pi*(j+0.5)*dy^2 ring.
real mid_section_area(const Case& cs, const Field& J, real x0, real y0, real dx, real dy) {
  const Config& C = cs.cfg;
  real F = 0;
  for (int j = 0; j < J.ny; j++) {
    bool hit = false;
    for (int i = 0; i < J.nx; i++) {
      const CellRecord& n = J.at(i, j);
      if ((n.is(CT_WALL_LAW) || n.is(CT_WALL_NO_SLIP)) && in_box(C, i, j, x0, y0, dx, dy)) hit = true;
    }
    if (hit) F += (C.FT == FT_FLAT) ? C.dy : 2 * M_PI * (j + 0.5) * C.dy * C.dy;
  }
  return F;
}

// SmoothX / SmoothY (out_cfd_param.cpp:500-522): in place, in the reference's
// j-outer / i-inner order, so a smoothed value feeds the next cell.
void smooth_y(real* A, int nx, int ny) {
  for (int j = 1; j < ny - 1; j++)
    for (int i = 0; i < nx; i++) {
      real* c = A + (size_t)i * ny;
      if (c[j + 1] > 0. && c[j - 1] > 0.) c[j] = 0.5 * (c[j + 1] + c[j - 1]);
    }
}
void smooth_x(real* A, int nx, int ny) {
  for (int j = 0; j < ny; j++)
    for (int i = 1; i < nx - 1; i++) {
      real& c = A[(size_t)i * ny + j];
      const real l = A[(size_t)(i - 1) * ny + j], r = A[(size_t)(i + 1) * ny + j];
      if (r > 0. && l > 0.) c = 0.5 * (r + l);
    }
}

void wall_span_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                     std::vector<real>& t) {
  const Config& C = cs.cfg;
  for (int i = ib; i < ie; i++) {
    bool hit = false;
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& n = J.at(i, j);
      if ((n.is(CT_WALL_LAW) || n.is(CT_WALL_NO_SLIP)) && in_box(C, i, j, x0, y0, dx, dy)) hit = true;
    }
    if (hit) t.push_back(C.dx);
  }
}

real body_pmax(real span, const GasFlow& f) { return f.ROG() * f.Wg2d() * f.Wg2d() * 0.5 * span; }

real calc_cx(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, const GasFlow& f) {
  std::vector<real> t;
  wall_span_terms(cs, J, x0, y0, dx, dy, 0, J.nx, t);
  const real Pmax = body_pmax(fold_terms(t), f);
  return Pmax == 0. ? 0 : x_force(cs, J, x0, y0, dx, dy) / Pmax;
}
real calc_cy(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, const GasFlow& f) {
  std::vector<real> t;
  wall_span_terms(cs, J, x0, y0, dx, dy, 0, J.nx, t);
  const real Pmax = body_pmax(fold_terms(t), f);
  return Pmax == 0. ? 0 : y_force(cs, J, x0, y0, dx, dy) / Pmax;
}
real calc_cp(const CellRecord& n, const GasFlow& f) {
  if (n.is(CT_WALL_NO_SLIP)) return (n.p - f.Pg()) / (0.5 * f.ROG() * f.Wg2d() * f.Wg2d());
  return 0;
}
real calc_cd(const Case& cs, const Field& J, real x0, real y0, real dy, const GasFlow& f) {
  return mass_flow_rate_x(cs, J, x0, y0, dy) / f.ROG() / f.Wg2d() / calc_area(cs, J, x0, y0, dy);
}
real calc_cv(const Case& cs, const Field& J, real x0, real y0, real dy, real p_amb, const GasFlow& f) {
  const Config& C = cs.cfg;
  const unsigned i = (unsigned)(x0 / C.dx);
  const unsigned j0 = (unsigned)(y0 / C.dy), j1 = (unsigned)((y0 + dy) / C.dy);
  real Fv = 0;
  if ((int)i >= J.nx) return 0;
  for (int j = (int)j0; j < (int)j1 && j < J.ny; j++) {
    const CellRecord& n = J.at(i, j);
    if (n.is(CT_SOLID)) continue;
    const real t = n.S[I_RHOU] * n.U + (n.p - p_amb);
    Fv += (C.FT == FT_FLAT) ? C.dy * t : 2 * M_PI * C.dy * n.y * t;
  }
  const real Mp = mass_flow_rate_x(cs, J, x0, y0, dy);
  return Mp > 0.0 ? Fv / (f.U() * Mp) : 0;
}

real average_pressure(const Case& cs, const Field& J, real x0, real l, real d) {
  const Config& C = cs.cfg;
  real pm = 0, Vs = 0;
  long n = 0;
  for (int i = 0; i < J.nx; i++)
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& c = J.at(i, j);
      if (c.is(CT_SOLID) || !(i > (int)(x0 / C.dx) && i < (int)((l + x0) / C.dx) && j < (int)(d / C.dy))) continue;
      if (C.FT == FT_AXISYMMETRIC) {
        const real Vi = 2 * M_PI * c.y * C.dy * C.dx;
        Vs += Vi;
        pm += c.p * Vi;
      } else {
        pm += c.p;
      }
      n++;
    }
  if (!n) return 0.;
  return C.FT == FT_AXISYMMETRIC ? pm / Vs : pm / n;
}

real average_temperature(const Case& cs, const Field& J, real x0, real l, real d, int mid_enthalpy) {
  const Config& C = cs.cfg;
  real Tm = 0, Vs = 0;
  long n = 0;
  for (int i = 0; i < J.nx; i++)
    for (int j = 0; j < J.ny; j++) {
      const CellRecord& c = J.at(i, j);
      if (c.is(CT_SOLID) || !(i > (int)(x0 / C.dx) && i < (int)((l + x0) / C.dx) && j < (int)(d / C.dy))) continue;
      if (C.FT == FT_AXISYMMETRIC) {
        real Vi = 2 * M_PI * c.y * C.dy * C.dx;
        if (mid_enthalpy) Vi *= c.CP;
        Vs += Vi;
        Tm += c.Tg * Vi;
      } else {
        Tm += c.Tg;
      }
      n++;
    }
  if (!n) return 0.;
  return C.FT == FT_AXISYMMETRIC ? Tm / Vs : Tm / n;
}

static real near_lam(const Field& J, int i, int j, const CellRecord& n, int& cnt) {
  const int N1 = i - n.idXl, N2 = i + n.idXr, N3 = j + n.idYu, N4 = j - n.idYd;
  real s = n.lam + n.lam_t;
  cnt = 5;
  s += J.at(N1, j).lam + J.at(N1, j).lam_t;
  s += J.at(N2, j).lam + J.at(N2, j).lam_t;
  s += J.at(i, N3).lam + J.at(i, N3).lam_t;
  s += J.at(i, N4).lam + J.at(i, N4).lam_t;
  return s;
}

bool heat_flux_x_cols(const Case& cs, const Field& J, int ib, int ie, real* Q, real* Al, real* Cp, real* St) {
  const Config& C = cs.cfg;
  if (C.Cp_Flow_index < 1 || C.Cp_Flow_index > (int)cs.flows2d.size()) return false;
  const GasFlow& F = cs.flows2d[C.Cp_Flow_index - 1];
  const real Trec = (1 + 0.45 * (F.kg() - 1.0) * F.flow_MACH() * F.flow_MACH()) * F.Tg();
  for (int i = ib; i < ie; i++) {
    // the reference also keeps laminar-correlation maxima (QR, AR) and Re, Pr
    // for its _REF_TEST_ build; only the written columns are formed here
    Q[i] = Al[i] = Cp[i] = St[i] = 0.;
    for (int j = std::max(0, C.y_min); j < std::min(C.y_max, J.ny - 1); j++) {
      const CellRecord& n = J.at(i, j);
      if (!n.is(CT_WALL_NO_SLIP)) continue;
      int cnt;
      const real lam_eff = near_lam(J, i, j, n, cnt) / cnt;
      real q = lam_eff * (n.Tg - C.Ts0) / C.dy;
      real alpha = lam_eff / C.dy;
      const real st = q / (F.ROG() * F.Wg2d() * F.C * (Trec - C.Ts0));
      const real cp = calc_cp(n, F);
      if (Q[i] != 0.) {
        Q[i] = std::max(Q[i], q);
        Al[i] = std::max(Al[i], alpha);
      } else {
        Q[i] = q;
        Al[i] = alpha;
      }
      Cp[i] = cp;
      St[i] = st;
    }
  }
  return true;
}

void write_x_heat_flux(const std::string& path, const Config& C, bool valid, const real* Q, const real* Al,
                       const real* Cp, const real* St) {
  std::ofstream o(path, std::ios::trunc);
  o << "#VARIABLES = X, HeatFlux(X),  Alpha(X), Cp(X), St(X)\n";
  if (!valid) return;
  // the reference's default build (no _REF_TEST_) writes X, Q, alpha, Cp, St
  for (int i = 0; i < C.MaxX; i++) o << i * C.dx << " " << Q[i] << " " << Al[i] << " " << Cp[i] << " " << St[i] << "\n";
}

void save_x_heat_flux(const std::string& path, const Case& cs, const Field& J) {
  const int NX = J.nx;
  std::vector<real> Q(NX, 0.), Al(NX, 0.), Cp(NX, 0.), St(NX, 0.);
  const bool ok = heat_flux_x_cols(cs, J, 0, NX, Q.data(), Al.data(), Cp.data(), St.data());
  write_x_heat_flux(path, cs.cfg, ok, Q.data(), Al.data(), Cp.data(), St.data());
}

void heat_flux_y_terms(const Case& cs, const Field& J, int ib, int ie, std::vector<real>& jq) {
  const Config& C = cs.cfg;
  for (int j = 0; j < J.ny; j++)
    for (int i = ib; i < std::min(ie, J.nx - 1); i++) {
      const CellRecord& n = J.at(i, j);
      if (!n.is(CT_WALL_NO_SLIP)) continue;
      int cnt;
      const real lam_eff = near_lam(J, i, j, n, cnt) / cnt;
      jq.push_back((real)j);
      jq.push_back(lam_eff * (n.Tg - C.Ts0) / C.dx);
    }
}

void fold_heat_flux_y(std::vector<real>& Q, const std::vector<real>& jq) {
  for (size_t k = 0; k + 1 < jq.size(); k += 2) {
    real& Qj = Q[(size_t)jq[k]];
    const real q = jq[k + 1];
    Qj = (Qj != 0.) ? std::max(Qj, q) : q;
  }
}

void write_y_heat_flux(const std::string& path, const Config& C, const std::vector<real>& Q) {
  std::ofstream o(path, std::ios::trunc);
  o << "#VARIABLES = Y, HeatFlux(Y)\n";
  for (int j = 0; j < C.MaxY; j++) o << j * C.dy << " " << Q[j] << "\n";
}

void save_y_heat_flux(const std::string& path, const Case& cs, const Field& J) {
  std::vector<real> jq, Q(J.ny, 0.);
  heat_flux_y_terms(cs, J, 0, J.nx, jq);
  fold_heat_flux_y(Q, jq);
  write_y_heat_flux(path, cs.cfg, Q);
}

namespace {
struct FlagName {
  u64 bit;
  const char* name;
};
const FlagName CT_NAMES[] = {
    {CT_Rho_CONST, "CT_Rho_CONST_2D"}, {CT_U_CONST, "CT_U_CONST_2D"}, {CT_V_CONST, "CT_V_CONST_2D"},
    {CT_T_CONST, "CT_T_CONST_2D"}, {CT_Y_CONST, "CT_Y_CONST_2D"}, {CT_dRhodx_NULL, "CT_dRhodx_NULL_2D"},
    {CT_dUdx_NULL, "CT_dUdx_NULL_2D"}, {CT_dVdx_NULL, "CT_dVdx_NULL_2D"}, {CT_dTdx_NULL, "CT_dTdx_NULL_2D"},
    {CT_dYdx_NULL, "CT_dYdx_NULL_2D"}, {CT_dRhody_NULL, "CT_dRhody_NULL_2D"}, {CT_dUdy_NULL, "CT_dUdy_NULL_2D"},
    {CT_dVdy_NULL, "CT_dVdy_NULL_2D"}, {CT_dTdy_NULL, "CT_dTdy_NULL_2D"}, {CT_dYdy_NULL, "CT_dYdy_NULL_2D"},
    {CT_d2Rhodx2_NULL, "CT_d2Rhodx2_NULL_2D"}, {CT_d2Udx2_NULL, "CT_d2Udx2_NULL_2D"},
    {CT_d2Vdx2_NULL, "CT_d2Vdx2_NULL_2D"}, {CT_d2Tdx2_NULL, "CT_d2Tdx2_NULL_2D"},
    {CT_d2Ydx2_NULL, "CT_d2Ydx2_NULL_2D"}, {CT_d2Rhody2_NULL, "CT_d2Rhody2_NULL_2D"},
    {CT_d2Udy2_NULL, "CT_d2Udy2_NULL_2D"}, {CT_d2Vdy2_NULL, "CT_d2Vdy2_NULL_2D"},
    {CT_d2Tdy2_NULL, "CT_d2Tdy2_NULL_2D"}, {CT_d2Ydy2_NULL, "CT_d2Ydy2_NULL_2D"},
    {CT_NONREFLECTED, "CT_NONREFLECTED_2D"}, {CT_WALL_NO_SLIP, "CT_WALL_NO_SLIP_2D"},
    {CT_WALL_LAW, "CT_WALL_LAW_2D"}, {CT_GAS, "CT_GAS_2D"}, {CT_BL_REFINEMENT, "CT_BL_REFINEMENT_2D"},
    {CT_SOLID, "CT_SOLID_2D"}, {CT_NODE_IS_SET, "CT_NODE_IS_SET_2D"}, {CT_LIQUID, "CT_LIQUID_2D"},
    {CT_TIME_DEPEND, "CT_TIME_DEPEND_2D"},
};
const FlagName TCT_NAMES[] = {
    {TCT_k_CONST, "TCT_k_CONST_2D"}, {TCT_eps_CONST, "TCT_eps_CONST_2D"}, {TCT_dkdx_NULL, "TCT_dkdx_NULL_2D"},
    {TCT_depsdx_NULL, "TCT_depsdx_NULL_2D"}, {TCT_dkdy_NULL, "TCT_dkdy_NULL_2D"},
    {TCT_depsdy_NULL, "TCT_depsdy_NULL_2D"}, {TCT_d2kdx2_NULL, "TCT_d2kdx2_NULL_2D"},
    {TCT_d2epsdx2_NULL, "TCT_d2epsdx2_NULL_2D"}, {TCT_d2kdy2_NULL, "TCT_d2kdy2_NULL_2D"},
    {TCT_d2epsdy2_NULL, "TCT_d2epsdy2_NULL_2D"}, {TCT_k_eps_Model, "TCT_k_eps_Model_2D"},
    {TCT_Prandtl_Model, "TCT_Prandtl_Model_2D"}, {TCT_Integral_Model, "TCT_Integral_Model_2D"},
    {TCT_eps_mud2kdx2_WALL, "TCT_eps_mud2kdx2_WALL_2D"}, {TCT_eps_mud2kdy2_WALL, "TCT_eps_mud2kdy2_WALL_2D"},
    {TCT_eps_Cmk2kXn_WALL, "TCT_eps_Cmk2kXn_WALL_2D"}, {TCT_Spalart_Allmaras_Model, "TCT_Spalart_Allmaras_Model_2D"},
    {TCT_k_omega_Model, "TCT_k_omega_Model_2D"}, {TCT_k_omega_SST_Model, "TCT_k_omega_SST_Model_2D"},
    {TCT_Baldwin_Lomax_Model, "TCT_Baldwin_Lomax_Model_2D"}, {TCT_nut_92_Model, "TCT_nut_92_Model_2D"},
    {TCT_Smagorinsky_Model, "TCT_Smagorinsky_Model_2D"},
};
template <size_t M>
std::string names(u64 v, const FlagName (&tab)[M], const char* none) {
  std::string s;
  for (const FlagName& f : tab)
    if ((v & f.bit) == f.bit) s += (s.empty() ? "" : " | ") + std::string(f.name);
  return s.empty() ? none : s;
}
}  // namespace

std::string cond_names(u64 CT) { return names(CT, CT_NAMES, "CT_NO_COND_2D"); }
std::string turb_cond_names(u64 TT) { return names(TT, TCT_NAMES, "TCT_No_Turbulence_2D"); }

}  // namespace hf2d
