// Output writers and integral post-processing on a host Field.
//   Tecplot/GNUPlot field file   SaveData2D     deeps2d_core.cpp:2589-2673
//   RMS / monitor files          SaveRMS*, SaveMonitors*  deeps2d_core.cpp:2532-2587
//   libOutCFD integrals          libOutCFD/out_cfd_param.cpp:14-809
// Formatting uses iostream defaults (6 significant digits) like the reference.
#pragma once

#include <ostream>
#include <string>
#include <vector>

#include "case.hpp"
#include "residual.hpp"

namespace hf2d {

// Field snapshot: rewrite (GNUPlot, blank line per j-row) or append (Tecplot).
void save_field_plt(const std::string& path, const Case& cs, const Field& J, real global_time, bool rewrite);
// the same for columns [ib, ie) only (a strip rank's error snapshot)
void save_field_plt_cols(const std::string& path, const Case& cs, const Field& J, real global_time, bool rewrite,
                         int ib, int ie);
// building blocks of the snapshot (stripio.cpp writes it without a gather)
std::string plt_header(const Case& cs, real global_time, int ncols);
const GasFlow* plt_cx_flow(const Case& cs);
void plt_row(std::ostream& o, const Case& cs, const Field& J, int j, int ib, int ie, const GasFlow* cxf);
void save_rms_header(const std::string& path, const Config& C);
// cd_cv: {Cd, Cv} of the nozzle cut when Cd output is on (else nullptr)
void append_rms(const std::string& path, long n, const real* rms, const Config& C, const real* cd_cv);
void save_monitors_header(const std::string& path, const Config& C);
void append_monitors(const std::string& path, real t, const std::vector<MonitorPoint>& m);
void save_x_heat_flux(const std::string& path, const Case& cs, const Field& J);
void save_y_heat_flux(const std::string& path, const Case& cs, const Field& J);
// heat-flux building blocks over columns [ib, ie): the per-column X arrays
// (false: no valid Cp flow, header only) and the Y terms as (j, q) pairs in
// the reference's (j, i) order, folded with its max-or-first rule
bool heat_flux_x_cols(const Case& cs, const Field& J, int ib, int ie, real* Q, real* Al, real* Cp, real* St);
void write_x_heat_flux(const std::string& path, const Config& C, bool valid, const real* Q, const real* Al,
                       const real* Cp, const real* St);
void heat_flux_y_terms(const Case& cs, const Field& J, int ib, int ie, std::vector<real>& jq);
void fold_heat_flux_y(std::vector<real>& Q, const std::vector<real>& jq);
void write_y_heat_flux(const std::string& path, const Config& C, const std::vector<real>& Q);

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
// Body integrals as ordered term lists over columns [ib, ie): the pressure and
// friction accumulators and the wall span, in the reference's (i, j) order.
// Folding the concatenated lists of all strips left to right reproduces the
// serial sums bit for bit.
void x_force_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                   std::vector<real>& fp, std::vector<real>& fd);
void y_force_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                   std::vector<real>& fp, std::vector<real>& fd);
void wall_span_terms(const Case& cs, const Field& J, real x0, real y0, real dx, real dy, int ib, int ie,
                     std::vector<real>& t);
real fold_terms(const std::vector<real>& t);
real body_pmax(real span, const GasFlow& f);
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
