// K12 kinetics for runtime (file) mechanisms on the MFMA matrix cores; see chem_mech.hip.
#pragma once
#include <memory>
#include <vector>

#include "../core/common.hpp"

struct ihipStream_t;   // hipStream_t, without pulling HIP headers into host-only units

namespace hf2d {

struct MechData;

// Device image of a mechanism (chem_mech_pack); R padded to a multiple of 16.
struct ChemMechDev {
  const double* nmat = nullptr;     // [16][R] nu'' - nu'
  const double* arr = nullptr;      // [3][R] A (SI), b, Ta = Ea/Ru
  const double* fall = nullptr;     // [7][R] A0, b0, Ta0, Troe a, T3, T1, T2
  const double* eff = nullptr;      // [R][16] collider efficiencies (third-body / fall-off steps)
  const double* thermo = nullptr;   // NASA-7 [16][2][7], then Tmid[16]
  const double* W = nullptr;        // [16] kg/mol
  const int* rx = nullptr;          // [R][4]: packed reactants, packed products (3 x (species | order << 4)
                                    //   << 6t), flags (rev | tb << 1 | fall-off << 2 | ntroe << 3 | (dnu + 16) << 8)
  int ns = 0, R = 0;
};

struct ChemMechPack {
  ChemMechDev dev;
  std::vector<void*> bufs;
  ~ChemMechPack();
};
std::unique_ptr<ChemMechPack> chem_mech_pack(const MechData& md);

// Cells [c0, c1) of species-major SoA arrays (stride N): S holds rho, rhoU,
// rhoV, rhoE (equation-major, stride N); Yin -> Yout; Tprev is the previous
// temperature (Newton start and the ChemTmin test); CT (optional) the cell
// flags (inactive cells copy through).
struct MechCells {
  const double* S = nullptr;
  const double* Yin = nullptr;
  double* Yout = nullptr;
  const double* Tprev = nullptr;
  double* Tout = nullptr;
  const u64* CT = nullptr;
  long N = 0, c0 = 0, c1 = 0;
  double Tchem = 0.0;
  // solver launches: the step's dt is read on the device from this slot
  // (IEEE bits of a positive double) instead of the dt argument
  const unsigned long long* dt_bits = nullptr;
  HF_HD bool active(long c) const {
    if (!CT) return true;
    const u64 ct = CT[c];
    return has_all(ct, CT_NODE_IS_SET) && !has_all(ct, CT_SOLID) && !has_all(ct, NT_FC);
  }
};

int chem_mech_max_reactions();
int chem_mech_launch(const ChemMechDev& m, const MechCells& q, double dt, int nsub, ihipStream_t* stream);

// Standalone operator: rhoY [ns][n] and T updated in place at constant (rho, e).
// Returns the mean kernel time in ms over `repeats` runs from the same input.
// valu: the same operator on the vector ALUs from the same runtime data
// (hf2d_chem_rt_valu: core/mechanism.hpp mech_chem_cell, one cell per lane) --
// the equal-terms baseline of the MFMA kernel (PARITY.md, K12).
double chem_mech_run_host(const MechData& md, double* rhoY, const double* rho, const double* e, double* T, long n,
                          double dt, int nsub, int repeats, bool valu = false);

}  // namespace hf2d
