// K12 kinetics for mechanisms loaded from a file: the compiled-mechanism
// kernels of chem_fast_dev.hpp, specialised at run time with hiprtc for the
// loaded mechanism (chem_rtc.hip).  A built-in mechanism has its kernels
// compiled into the library (chem_fast.hip); any other mechanism gets the same
// register-resident integrator after a one-time compile whose code object is
// cached on disk, instead of the runtime-data MFMA kernel.
#pragma once
#include <string>

struct ihipStream_t;

namespace hf2d {

struct MechData;
struct SoA;
struct DevScalars;

// The constexpr mechanism struct (`MechRtc`) the kernels are instantiated for,
// generated from the runtime mechanism data (the C++ counterpart of
// tools/gen_mech_header.py).
std::string mech_struct_source(const MechData& m, const std::string& name = "MechRtc");
// Full hiprtc translation unit (headers inlined) for mechanism m.
std::string chem_rtc_program(const MechData& m);

// Compile (or load from the cache) the kernels of mechanism m.  False (with
// *why) when hiprtc fails; the caller falls back to the runtime-data kernel.
bool chem_rtc_prepare(const MechData& m, std::string* why);
// mechanism-mode kinetics of cells [c0, c1) with the prepared kernels
// (compacted form when list / count are given; list_ready: the list and its
// count are already built on the device, only the listed cells are integrated
// in place -- the lean mechanism step, hip/lean_mech.hpp)
bool chem_rtc_launch(const MechData& m, const SoA& mid, const SoA& out, const double* Tprev, long c0, long c1,
                     DevScalars* sc, int slot, double Tchem, int nsub, ihipStream_t* st, int* list, unsigned* count,
                     bool list_ready = false);
// standalone operator on n cells (rhoY [ns][n] and T in place); mean kernel ms
double chem_rtc_run_host(const MechData& m, double* rhoY, const double* rho, const double* e, double* T, long n,
                         double dt, int nsub, int repeats);
// hiprtc compile (or cache hit) only, no device needed: code object bytes, -1 on failure
long chem_rtc_compile(const MechData& m, std::string* why, bool* cached);
// where compiled code objects are cached, and whether the last prepare hit it
std::string chem_rtc_cache_dir();
bool chem_rtc_last_cached();

}  // namespace hf2d
