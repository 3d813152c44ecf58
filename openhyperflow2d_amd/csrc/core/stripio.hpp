// Outputs of a strip-decomposed run without a full-field gather.
//
// The reference funnels every output through rank 0: at each cycle end the
// sub-domains are received whole by rank 0 (deeps2d_core.cpp:1695-1745,
// LongMatrixRecv) before the Cut/Cx lines (1760-1815), SaveData2D and the
// swap file.  Here each rank keeps and
// downloads only its strip (plus one ghost column each side) and
//   * formats its share of every Tecplot row and pwrites it at an offset
//     computed from the all-gathered row lengths (rank 0 writes the header);
//   * pwrites its column range of the .hf2d image (x-major records, one
//     contiguous byte range per strip);
//   * evaluates the integrals over its own columns as ordered term lists
//     (postproc.hpp) that are all-gathered and folded left to right, so the
//     Cut / Cx / Cd / heat-flux values are bit-identical to one rank.
// Every function is collective over `comm` (all ranks call it, same order).
#pragma once

#include <string>
#include <vector>

#include "case.hpp"
#include "solver.hpp"

namespace hf2d {

// the neighbours' first/last owned columns into this rank's ghost columns
void strip_exchange_ghosts(Comm& comm, Field& J, int gi0, int gi1);
// field snapshot (rewrite: GNUPlot blank line per row; else Tecplot append)
void strip_write_plt(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1,
                     real global_time, bool rewrite);
// .hf2d checkpoint image: rank 0 sizes the file, every rank writes its columns
void strip_write_hf2d(Comm& comm, const std::string& path, const Field& J, int gi0, int gi1);
// the value of the one rank that has it (have = owns the cut column), else 0
real strip_pick(Comm& comm, bool have, real v);
// per-list sums of the rank-ordered concatenation of each rank's term lists
std::vector<real> strip_fold(Comm& comm, const std::vector<std::vector<real>>& lists);

// Driver-level outputs (solver.cpp run_cycles), all collective:
real strip_mass_flow(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, real x0, real y0, real dy);
// {Cd, Cv} of the nozzle cut (append_rms)
void strip_cd_cv(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, const GasFlow& f, real out[2]);
// {Cx, Cy, Fx, Fy} of the body box
void strip_body_forces(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, const GasFlow& f, real out[4]);
// HeatFlux-X / HeatFlux-Y files (written by rank 0)
void strip_heat_flux_x(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1);
void strip_heat_flux_y(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1);

}  // namespace hf2d
