// Output writers and integral post-processing on a host Field.
//   Tecplot/GNUPlot field file   SaveData2D     deeps2d_core.cpp:2589-2673
//   RMS / monitor files          SaveRMS*, SaveMonitors*  deeps2d_core.cpp:2532-2587
//   libOutCFD integrals          libOutCFD/out_cfd_param.cpp:14-809
// Formatting uses iostream defaults (6 significant digits) like the reference.
#pragma once

#include <ostream>
#include <string>

#include "case.hpp"
#include "residual.hpp"

namespace hf2d {

// Field snapshot: rewrite (GNUPlot, blank line per j-row) or append (Tecplot).
void save_field_plt(const std::string& path, const Case& cs, const Field& J, real global_time, bool rewrite);
void save_rms_header(const std::string& path, const Config& C);
void append_rms(const std::string& path, long n, const real* rms, const Case& cs, const Field& J);
void save_monitors_header(const std::string& path, const Config& C);
void append_monitors(const std::string& path, real t, const std::vector<MonitorPoint>& m);
void save_x_heat_flux(const std::string& path, const Case& cs, const Field& J);
void save_y_heat_flux(const std::string& path, const Case& cs, const Field& J);

// libOutCFD
real p_asterisk(const CellRecord& n);
real T_asterisk(const CellRecord& n);
real schlieren(const CellRecord& n);
real re_airfoil(real chord, const GasFlow& f);
real mass_flow_rate_x(const Case& cs, const Field& J, real x0, real y0, real dy);
real calc_area(const Case& cs, const Field& J, real x0, real y0, real dy);
real x_force(const Case& cs, const Field& J, real x0, real y0, real dx, real dy);
real y_force(const Case& cs, const Field& J, real x0, real y0, real dx, real dy);
real x_force_ysym(const Case& cs, const Field& J, real x0, real l, real d);
real mid_section_area(const Case& cs, const Field& J, real x0, real y0, real dx, real dy);
void smooth_x(real* A, int nx, int ny);   // x-major (nx, ny) array, in place
void smooth_y(real* A, int nx, int ny);
real calc_cx(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, const GasFlow& f);
real calc_cy(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, const GasFlow& f);
real calc_cp(const CellRecord& n, const GasFlow& f);
real calc_cd(const Case& cs, const Field& J, real x0, real y0, real dy, const GasFlow& f);
real calc_cv(const Case& cs, const Field& J, real x0, real y0, real dy, real p_amb, const GasFlow& f);
real average_pressure(const Case& cs, const Field& J, real x0, real l, real d);
real average_temperature(const Case& cs, const Field& J, real x0, real l, real d, int mid_enthalpy);

// PrintCond / PrintTurbCond (deeps2d_core.cpp:2390-2491): names of the set
// CondType2D / TurbulenceCondType2D bits, e.g. "CT_U_CONST_2D | CT_NODE_IS_SET_2D".
std::string cond_names(u64 CT);
std::string turb_cond_names(u64 TT);

}  // namespace hf2d
