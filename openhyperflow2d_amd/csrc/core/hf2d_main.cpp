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
//     --transport p2p|rccl    multi-GPU halo transport (default p2p, RCCL fallback)
//     --reference-exit-status exit 0 after a Tg < 0 abort, as the reference does
//                             (Abort_OpenHyperFLOW2D, hyper_flow_area.cpp:17-33);
//                             by default such a run exits 1
//
// Multi-process runs (one rank per GPU, or per CPU strip): RANK, WORLD_SIZE,
// LOCAL_RANK, MASTER_ADDR, MASTER_PORT as torchrun or bin/OpenHyperFLOW2D.sh
// set them.  The ranks meet over TCP at rank 0 (tcpcomm.hpp), cut the grid
// into balanced strips and run the same driver; every rank writes its share
// of the outputs (stripio.hpp).  The reference does the same with MPI inside
// main (hf2d_start.cpp:79-289).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>

#include "case.hpp"
#include "solver.hpp"
#include "tcpcomm.hpp"

namespace hf2d {
// Implemented in hip/device_solver.hip when the GPU backend is linked in.
std::unique_ptr<SolverBase> make_gpu_solver(Case& cs, int device) __attribute__((weak));
std::unique_ptr<SolverBase> make_gpu_strip_solver(Case& cs, int device, int gi0, int gi1, Comm& boot,
                                                  const std::string& transport, std::string& used)
    __attribute__((weak));
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
  std::string backend, deck_path, outdir = ".", profile, fault_kind = "nan", transport = "p2p";
  int cycles = -1, device = -1, fault_rank = 0;
  long fault_step = -1;
  bool serial = false, use_ckpt = true, ref_exit = false;
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
    else if (s == "--fault-rank" && a + 1 < argc) fault_rank = std::atoi(argv[++a]);
    else if (s == "--transport" && a + 1 < argc) transport = argv[++a];
    else if (s == "--reference-exit-status") ref_exit = true;
    else deck_path = s;
  }
  const RankEnv env = RankEnv::from_environ();
  const bool root = env.rank == 0;
  std::ostringstream quiet;
  std::ostream& out = root ? std::cout : quiet;   // banner / pre-processor log: rank 0
  try {
    std::unique_ptr<TcpComm> tcp;
    if (env.world > 1) tcp.reset(new TcpComm(env.rank, env.world, env.addr, env.port));
    InputDeck deck = InputDeck::from_file(deck_path);
    out << "Load \"" << deck.name() << "\" data...OK\n";
    if (device < 0) {
      device = deck.get_int_or("isSingleGPU", 0) ? deck.get_int_or("ActiveSingleGPU", 0) : 0;
      if (env.world > 1) device = env.local_rank;   // one GPU per local rank
    }
    // Multi-rank: strip-local pre-processing, no whole field anywhere (SURVEY
    // 5.7; the reference's rank 0 pre-processes all of it and scatters,
    // hf2d_start.cpp:143-205): every rank cuts the strips from a flags-only
    // pass, pre-processes its own columns + one ghost column each side on the
    // whole grid's 16 B/cell flag plane (a restart reads its slab of the
    // .hf2d), and the whole-field eligibility facts are gathered from every
    // strip in rank order
    Case cs;
    std::vector<std::pair<int, int>> parts;
    if (env.world > 1) {
      parts = Case::partition_deck(deck, outdir, use_ckpt, env.world);
      const int a = parts[env.rank].first, b = parts[env.rank].second;
      cs = Case::from_deck_window(deck, outdir, use_ckpt, std::max(a - 1, 0), std::min(b + 1, parts.back().second),
                                  root ? &std::cout : nullptr);
      if (serial) cs.cfg.semantics = Semantics::SERIAL;
      std::vector<FactsPart> fp;
      for (const std::string& blob : tcp->allgather_bytes(cs.facts_part().pack())) fp.push_back(FactsPart::unpack(blob));
      cs.merge_facts(fp);
    } else {
      cs = Case::from_deck(deck, outdir, use_ckpt, &std::cout);
      if (serial) cs.cfg.semantics = Semantics::SERIAL;
      parts = balanced_columns(cs.J, 1);
    }
    out << "X=" << cs.cfg.MaxX << "  Y=" << cs.cfg.MaxY << "  dx=" << cs.cfg.dx << "  dy=" << cs.cfg.dy << "\n";
    out << "\nInitial dt=" << cs.dt0 << "sec.\n";
    out << "\nSolver Mode: " << (cs.cfg.ProblemType == SM_NS ? "Navier-Stokes" : "Euler") << "/FP64\n\n";
    if (backend.empty()) backend = (gpu_available && gpu_available()) ? "gpu" : "cpu";
    const int gi0 = parts[env.rank].first, gi1 = parts[env.rank].second;
    std::unique_ptr<SolverBase> solver;
    std::string used = "none";
    if (backend == "ref") {
      if (env.world > 1) throw std::runtime_error("the reference-order backend runs on one rank");
      solver.reset(new RefSolver(cs));
    } else if (backend == "gpu") {
      if (!make_gpu_strip_solver) throw std::runtime_error("GPU backend not linked into this build");
      Comm single;
      solver = make_gpu_strip_solver(cs, device, gi0, gi1, tcp ? (Comm&)*tcp : single, transport, used);
    } else {
      CpuSolver* c = new CpuSolver(cs, gi0, gi1);
      solver.reset(c);
      if (tcp) {
        TcpComm* t = tcp.get();
        c->comm = t;
        // halo columns over the neighbour sockets (same packing as the gloo path)
        c->halo_exchange = [t](CpuSolver& s, int g) {
          const size_t n = (size_t)s.halo_doubles(g) * s.h.ny;
          const bool L = s.gi0 > 0, R = s.gi1 < s.cs.J.nx;
          std::vector<real> sl(L ? n : 0), rl(L ? n : 0), sr(R ? n : 0), rr(R ? n : 0);
          if (L) s.pack_column(g, s.l_off, sl.data());
          if (R) s.pack_column(g, s.l_off + (s.gi1 - s.gi0) - 1, sr.data());
          t->neighbor_exchange(sl.data(), rl.data(), L ? n * sizeof(real) : 0, sr.data(), rr.data(),
                               R ? n * sizeof(real) : 0);
          if (L) s.unpack_column(g, 0, rl.data());
          if (R) s.unpack_column(g, s.h.nx - 1, rr.data());
        };
        used = "tcp";
      }
    }
    if (env.world > 1) out << "Ranks: " << env.world << " strips, halo transport " << used << "\n";
    out << "Start computation (" << backend << " backend)...\n" << std::flush;
    install_signal_handlers();
    RunOptions opt;
    opt.max_cycles = cycles;
    opt.outdir = outdir;
    opt.profile_path = profile.empty() || env.world == 1 ? profile : profile + ".rank" + std::to_string(env.rank);
    opt.fault_step = fault_step;
    opt.fault_rank = fault_rank;
    opt.fault_kind = fault_kind;
    // rank 0 logs the run; the others report only their own failure
    solver->run(opt, &std::cout);
    out << "\nResults saved in file \"" << cs.cfg.out_file << "\".\n";
    out << "\nReady. Computation finished.\n";
  } catch (const std::exception& e) {
    std::cout << "\n" << (env.world > 1 ? "[rank " + std::to_string(env.rank) + "] " : std::string()) << e.what()
              << "\nComputation terminated.\n";
    if (ref_exit && std::strstr(e.what(), "unstability")) return 0;
    return 1;
  }
  return 0;
}
