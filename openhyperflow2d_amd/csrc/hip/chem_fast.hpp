// K12 kinetics with a compiled mechanism (chem_fast.hip).
#pragma once
#include <string>

struct ihipStream_t;   // hipStream_t, without pulling HIP headers into host-only units

namespace hf2d {

struct StepParams;
struct SoA;
struct DevScalars;

bool chem_fast_available(const std::string& mech);
// mechanism-mode step kernel over linear cells [c0, c1): mid.Ys -> out.Ys.
// list (>= c1 - c0 ints) + count: compacted form (reacting cells only do work);
// list_ready: list and count already built on the device (lean mechanism step)
bool chem_fast_launch(const std::string& mech, const StepParams& P, const SoA& mid, const SoA& out, const double* Tprev,
                      long c0, long c1, DevScalars* sc, int slot, double Tchem, int nsub, ihipStream_t* st,
                      int* list = nullptr, unsigned* count = nullptr, bool list_ready = false);
// standalone operator on n cells (rhoY [ns][n] and T updated in place); mean kernel ms
double chem_fast_run_host(const std::string& mech, double* rhoY, const double* rho, const double* e, double* T, long n,
                          double dt, int nsub, int repeats);

}  // namespace hf2d
