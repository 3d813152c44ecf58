// K12 finite-rate mechanism chemistry (MFMA FP64); see chem_mech.hip.
#pragma once
struct ihipStream_t;   // hipStream_t, without pulling HIP headers into host-only units

namespace hf2d {

struct ChemMechDev {
  const double* nmat = nullptr;   // [16][R] net stoichiometry nu'' - nu' (rows >= ns zero)
  const double* arr = nullptr;    // A[R] (SI), b[R], Ta[R] = Ea/Ru  ->  kf = A T^b exp(-Ta/T)
  const int* rsp = nullptr;       // [R][3] reactant species (< ns)
  const int* rord = nullptr;      // [R][3] reactant orders (0 = unused slot)
  const double* W = nullptr;      // [ns] molar masses [kg/mol]
  int ns = 0, R = 0;
};

int chem_mech_max_reactions();
int chem_mech_launch(const ChemMechDev& m, double* rhoY, const double* T, int ncell, double dt, int nsub,
                     ihipStream_t* stream);

// Host convenience: upload, run `repeats` times (each from the same input), download.
// Returns the mean kernel time in ms.
double chem_mech_run_host(const double* nmat, const double* arr, const int* rsp, const int* rord, const double* W,
                          int ns, int R, double* rhoY, const double* T, int ncell, double dt, int nsub, int repeats);

}  // namespace hf2d
