// hf2d — command-line driver, argv-compatible with "OpenHyperFLOW2D-<ver> <deck.dat>"
// (reference hf2d_start.cpp:32-368).  Without arguments it prints the banner.
//
//   hf2d [options] deck.dat
//     --backend cpu|ref|gpu   stepper (default: gpu if a device is present, else cpu)
//     --semantics mpi|serial  reference build to mimic (default mpi)
//     --cycles N              stop after N outer cycles
//     --no-checkpoint         ignore/skip <Project>.hf2d
//     --outdir DIR            output directory
//     --device N              GPU ordinal (deck keys isSingleGPU/ActiveSingleGPU also honoured)
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>

#include "case.hpp"
#include "solver.hpp"

namespace hf2d {
// Implemented in hip/device_solver.cpp when the GPU backend is linked in.
std::unique_ptr<SolverBase> make_gpu_solver(Case& cs, int device) __attribute__((weak));
bool gpu_available() __attribute__((weak));
}  // namespace hf2d

int main(int argc, char** argv) {
  using namespace hf2d;
  if (argc < 2) {
    std::printf("hf2d / OpenHyperFLOW2D-compatible DEEPS solver for AMD Instinct MI355X (FP%u)\n",
                (unsigned)(sizeof(real) * 8));
    std::printf("Usage: %s [options] [{input_data_file}]\n", argv[0]);
    std::printf("\n\t* Density-based 2D-Navier-Stokes solver for uniform cartesian mesh");
    std::printf("\n\n\tFlowNode2D size = %d bytes\n\n", (int)sizeof(CellRecord));
    return 0;
  }
  std::string backend, deck_path, outdir = ".", profile, fault_kind = "nan";
  int cycles = -1, device = -1;
  long fault_step = -1;
  bool serial = false, use_ckpt = true;
  for (int a = 1; a < argc; a++) {
    std::string s = argv[a];
    if (s == "--backend" && a + 1 < argc) backend = argv[++a];
    else if (s == "--semantics" && a + 1 < argc) serial = std::string(argv[++a]) == "serial";
    else if (s == "--cycles" && a + 1 < argc) cycles = std::atoi(argv[++a]);
    else if (s == "--no-checkpoint") use_ckpt = false;
    else if (s == "--outdir" && a + 1 < argc) outdir = argv[++a];
    else if (s == "--device" && a + 1 < argc) device = std::atoi(argv[++a]);
    else if (s == "--profile" && a + 1 < argc) profile = argv[++a];
    else if (s == "--fault-step" && a + 1 < argc) fault_step = std::atol(argv[++a]);
    else if (s == "--fault-kind" && a + 1 < argc) fault_kind = argv[++a];
    else deck_path = s;
  }
  try {
    InputDeck deck = InputDeck::from_file(deck_path);
    std::cout << "Load \"" << deck.name() << "\" data...OK\n";
    if (device < 0) device = deck.get_int_or("isSingleGPU", 0) ? deck.get_int_or("ActiveSingleGPU", 0) : 0;
    Case cs = Case::from_deck(deck, outdir, use_ckpt, &std::cout);
    if (serial) cs.cfg.semantics = Semantics::SERIAL;
    std::cout << "X=" << cs.cfg.MaxX << "  Y=" << cs.cfg.MaxY << "  dx=" << cs.cfg.dx << "  dy=" << cs.cfg.dy << "\n";
    std::cout << "\nInitial dt=" << cs.dt0 << "sec.\n";
    std::cout << "\nSolver Mode: " << (cs.cfg.ProblemType == SM_NS ? "Navier-Stokes" : "Euler") << "/FP64\n\n";
    if (backend.empty()) backend = (gpu_available && gpu_available()) ? "gpu" : "cpu";
    std::unique_ptr<SolverBase> solver;
    if (backend == "ref")
      solver.reset(new RefSolver(cs));
    else if (backend == "gpu") {
      if (!make_gpu_solver) throw std::runtime_error("GPU backend not linked into this build");
      solver = make_gpu_solver(cs, device);
    } else
      solver.reset(new CpuSolver(cs));
    std::cout << "Start computation (" << backend << " backend)...\n" << std::flush;
    install_signal_handlers();
    RunOptions opt;
    opt.max_cycles = cycles;
    opt.outdir = outdir;
    opt.profile_path = profile;
    opt.fault_step = fault_step;
    opt.fault_kind = fault_kind;
    solver->run(opt, &std::cout);
    std::cout << "\nResults saved in file \"" << cs.cfg.out_file << "\".\n";
    std::cout << "\nReady. Computation finished.\n";
  } catch (const std::exception& e) {
    std::cout << "\n" << e.what() << "\nComputation terminated.\n";
    return 1;
  }
  return 0;
}
