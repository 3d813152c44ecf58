// Mechanism loading and the versioned species checkpoint.
//
// The .hf2d image keeps the reference's 1248-byte FlowNode2D<double,3> record
// for every run (NUM_COMPONENTS = 3 files stay byte-identical).  A mechanism
// run adds the sidecar <Project>.hf2d.species (layout version 2):
//   bytes 0..7    magic "HF2DSPC2"
//   u32 version (2), u32 ns, u32 nx, u32 ny
//   ns x 16-byte species names (NUL padded)
//   nx*ny*ns doubles: rho*Y_s per cell, cells in the .hf2d (x-major) order,
//   so a strip of columns is one contiguous byte range (per-rank slab writes).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "mechanism.hpp"

namespace hf2d {

struct MechInfo {
  std::string name, source;
  std::vector<std::string> species;
  MechData data;
  const MechData* data_ptr() const { return &data; }
};

std::shared_ptr<MechInfo> parse_mechanism(const std::string& text);
// built-in name ("h2_air_li2004") or a *.mech path (relative to workdir first)
std::shared_ptr<MechInfo> load_mechanism(const std::string& name, const std::string& workdir = "");
// kinetics/thermo data identical (a file copy of a built-in mechanism may use its compiled kernel)
bool mech_same_kinetics(const MechData& a, const MechData& b);
bool mech_is_builtin(const MechInfo& m, const std::string& builtin);

constexpr size_t SPECIES_HEADER = 8 + 16;
size_t species_sidecar_bytes(int ns, int nx, int ny);
// rhoY is species-major [ns][nx*ny] (the solver's SoA layout)
void write_species_sidecar(const std::string& path, const MechInfo& m, int nx, int ny, const std::vector<real>& rhoY);
// columns [gi0, gi0 + ncols) of a species-major local array whose column 0 is
// global column col0 (per-rank slab write into an existing full-size file)
void write_species_slab(const std::string& path, const MechInfo& m, int nx, int ny, const real* rhoY_local,
                        long local_n, int local_i0, int gi0, int ncols);
// (a >= 0: only the columns [a, b), species-major over them)
bool read_species_sidecar(const std::string& path, const MechInfo& m, int nx, int ny, std::vector<real>& rhoY,
                          int a = -1, int b = -1);

// Tecplot Y_fuel / Y_ox / Y_cp / Y_i columns of a mechanism state: the
// dominant species of each reference slot, the rest lumped into Y_i.
HF_HD inline void mech_slot_fractions(const MechData& m, const real* Y, real* Y4) {
  real rest = 1.0;
  for (int k = 0; k < 3; k++) {
    const int s = m.slot_sp[k];
    Y4[k] = s >= 0 ? Y[s] : 0.0;
    rest -= Y4[k];
  }
  Y4[3] = rest;
}

}  // namespace hf2d
