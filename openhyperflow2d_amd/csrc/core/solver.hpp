// Solvers and the time-march driver.
//
//   SolverBase     the DEEPS2D_Run outer/inner loop (deeps2d_core.cpp:723-1884):
//                  scenario tables, dt bookkeeping, residual/monitor logging,
//                  per-cycle outputs, checkpointing and the exit monitor.
//   CpuSolver      Jacobi stepper over host SoA arrays; uses the same per-cell
//                  kernels as the GPU (stepkern.hpp).  Strip-aware: a rank owns
//                  columns [i0, i1) of a local array with halo columns.
//   RefSolver      reference-order (in-place, Gauss-Seidel-like) stepper on
//                  AoS records, used as the golden-comparison oracle against
//                  the reference binary.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <utility>
#include <string>
#include <vector>

#include "case.hpp"
#include "residual.hpp"
#include "lean_euler.hpp"

namespace hf2d {

struct StepResult {
  real dt_min = 1.0;        // min local dt of this step (before cross-rank reduction)
  int neg_T = 0;
  bool have_residual = false;
  bool async = false;       // device backend: dt / time / neg_T stay on the device
  ResidualPack res;
};

// Host SoA arrays (also the staging format for device upload/download).
struct HostArrays {
  int nx = 0, ny = 0;
  long N = 0;
  std::vector<real> S[2], A, B, F, Src, SrcAdd, beta, dSdx[2], dSdy[2];
  std::vector<real> U[2], V[2], Tg[2], p, kk, R, CP, lam, mu, mu_t, lam_t, Diff, Y;
  std::vector<real> l_min, y_plus, Re_local, BGX, BGY, Tf, Q_conv, grad, qdir;
  std::vector<u64> CT, TT;
  std::vector<uint8_t> nb;
  std::vector<uint8_t> gf;  // GF_* traffic flags (compute_generic_flags)
  std::vector<int32_t> wslot;       // cell -> its wall's index in Case::wall_nodes (-1 none)
  std::vector<long> wall_own;        // local index of each wall node this strip owns
  std::vector<int32_t> wall_own_slot;   // ... and its index in Case::wall_nodes
  std::vector<real> time;   // per-cell record time (checkpoint only)
  // mechanism mode (SK_MECH): species block, species-major [s * N + idx]
  int nsp = 0;
  const MechData* mech = nullptr;
  std::vector<real> Ys[2], As, Bs, Fs, betas, dSdxs[2], dSdys[2];
  void allocate_mech(const Case& cs);
  // species of columns [gi0, gi0 + nx) from Case::mech_rhoY (fluxes: inviscid)
  void mech_from_case(const Case& cs, int gi0);
  void mech_to_case(Case& cs, int gi0, int i_from, int i_to, int ybuf) const;

  void allocate(int X, int Y);
  // columns [gi0, gi0 + X) of J
  void from_field(const Field& J, int gi0);
  void to_field(Field& J, int gi0, int i_from, int i_to, int prim_buf, int ds_buf) const;
  SoA view(int sbuf, int dsbuf, int pbuf);
  // sets the species members of a view (ybuf: species state buffer)
  void mech_view(SoA& s, int ybuf, int dsbuf) const;
  // wslot / wall_own for columns [gi0, gi1) owned, local column 0 = global gx0
  void wall_slots(const Case& cs, int gx0, int gi0, int gi1);
};

// Communication hooks for multi-rank (strip) runs.  Single-rank: no-ops.
struct Comm {
  virtual ~Comm() = default;
  virtual int rank() const { return 0; }
  virtual int size() const { return 1; }
  virtual real allreduce_min(real v) { return v; }
  virtual void allreduce_residual(ResidualPack&) {}
  virtual int allreduce_max_int(int v) { return v; }
  virtual real allreduce_sum(real v) { return v; }
  // Variable-size all-gather: every rank receives every rank's bytes, in rank
  // order.  Carries the outputs of a strip run (stripio.hpp: row lengths,
  // ghost columns, integral terms) -- never a whole field.
  virtual std::vector<std::string> allgather_bytes(const std::string& mine) { return {mine}; }
  void barrier() {
    if (size() > 1) (void)allgather_bytes(std::string());
  }
};

struct RunOptions {
  int max_cycles = -1;       // stop after this many outer cycles (-1: exit monitor only)
  bool write_outputs = true;
  bool write_checkpoint = true;
  std::string outdir = ".";
  bool verbose = true;
  std::string metrics_path;  // non-empty: append one JSON line per output step (metrics.jsonl)
  // per-phase wall-clock profile (JSON written when run() returns or fails)
  std::string profile_path;
  // Fault injection (tests of the failure / restart paths): at global
  // iteration fault_step on rank fault_rank, "nan" poisons one active cell
  // (negative energy -> Tg < 0 -> error snapshot), "kill" raises SIGKILL.
  long fault_step = -1;
  int fault_rank = 0;
  std::string fault_kind = "nan";
};

class SolverBase {
 public:
  explicit SolverBase(Case& cs);
  virtual ~SolverBase() = default;

  Case& cs;
  // false: the backend may skip output-only fields on this step (the host
  // will not read the record before the next step)
  bool step_outputs = true;
  Comm* comm = nullptr;      // owned elsewhere
  Comm local_comm;
  real dt = 0;               // dt used by the next step
  real dt_running = 1.0;     // serial semantics: never reset
  // Config::LaggedDt: the MIN of the last step's local dts, used by the step
  // after next (<= 0: not yet set -- the next step's dt)
  real dt_lag = -1.0;
  long iter = 0;             // iteration inside the current cycle
  long last_iter = 0;        // completed iterations of previous cycles
  bool ckpt_written = false; // a cycle-end checkpoint of this run exists
  real cur_time_part = 0;
  int cycle = 0;
  ResidualSummary last_res{};
  bool last_res_valid = false;
  double step_seconds = 0;   // wall time of the last cycle

  // One iteration (inner loop body).  want_res forces the residual pass.
  StepResult advance(bool want_res);
  // n iterations without outputs (benchmarks / tests).
  void run_steps(long n, bool want_res_last = false);
  // Full DEEPS2D_Run driver.  Returns the number of cycles run.
  int run(const RunOptions& opt, std::ostream* log);
  void write_profile(const std::string& path, int cycles) const;

  // Backend interface
  virtual StepResult do_step(const StepParams& P, bool want_res) = 0;
  virtual void download(Field& J) = 0;   // refresh host records (owned columns)
  virtual void upload() = 0;             // host records -> backend
  virtual void cycle_update() {}         // per-cycle y+ / sources (backend side)
  virtual void sample_monitors(std::vector<MonitorPoint>& mp);
  // device backends: pull dt, accumulated time and the error flag to the host
  virtual void sync_scalars() {}
  // called after an outer-cycle roll-over (cur_time_part folded into global_time)
  virtual void on_cycle_roll() {}
  StepParams make_params(long it) const;
  // y+ across strips: every wall node's friction velocity from its owner
  // (slots/vals: this rank's gas wall nodes) -> uw/ok over Case::wall_nodes
  void merge_wall_uw(const std::vector<int32_t>& slots, const std::vector<real>& vals, std::vector<real>& uw,
                     std::vector<uint8_t>& ok);
  // Overwrite the energy of global cell (gi, j) (owned by this backend) with
  // a negative value: fault injection for the Tg < 0 failure path.
  virtual void poison_cell(int gi, int j) = 0;
  // Profiler ranges around driver phases (device backends: roctx).
  virtual void trace_push(const char*) {}
  virtual void trace_pop() {}
  // accumulated wall-clock seconds and entry count per driver phase
  std::map<std::string, std::pair<double, long>> phase_acc;
  // global columns [first, second) this backend owns (strip decomposition)
  virtual std::pair<int, int> owned_columns() const { return {0, cs.J.nx}; }

 protected:
  bool isSrcAdd = false;
  int run_cycles(const RunOptions& opt, std::ostream* log);
  void failure_snapshot(const RunOptions& opt, const std::string& dir, const std::string& why, std::ostream* log);
  void inject_fault(const RunOptions& opt);
};

// Graceful stop (SIGINT / SIGTERM): the driver finishes the current step,
// writes the cycle outputs and the checkpoint, then returns.  Multi-rank runs
// agree on the flag at the next output step.
void request_stop();
bool stop_requested();
void clear_stop();
void install_signal_handlers();

// lean inviscid path (lean.cpp)
bool lean_eligible(const Case& cs, std::string* why);
bool lean_single_gas(const Case& cs);
int sk_eligible(const Case& cs, std::string* why);   // SK_* mode of the split kernels
bool lean_any_cauchy_x(const Case& cs);
bool mech_species_cauchy(const Case& cs);   // some node applies d2(rhoY)/dx2 or /dy2 = 0
// per-cell GF_* flags of the generic stepper (from the uploaded host arrays)
void compute_generic_flags(const Case& cs, HostArrays& h, int gx0);
std::vector<uint8_t> lean_flags(const HostArrays& h, int sm);

class CpuSolver : public SolverBase {
 public:
  // Owns columns [gi0, gi1) of the global field; a halo column is added on
  // each interior side.
  CpuSolver(Case& cs, int gi0 = 0, int gi1 = -1);
  StepResult do_step(const StepParams& P, bool want_res) override;
  std::pair<int, int> owned_columns() const override { return {gi0, gi1}; }
  void download(Field& J) override;
  void upload() override;
  void cycle_update() override;
  void poison_cell(int gi, int j) override;

  HostArrays h;
  int gi0, gi1;     // owned global columns
  int l_off;        // local index of global column gi0 (0 or 1)
  int sbuf = 0, dsbuf = 0, pbuf = 0;
  // halo access for distributed runs: pack/unpack columns of the exchanged fields
  // groups: 0 = predicted state (N-S gradients), 1 = post-fill state,
  // 2 = wall-heat per-direction fluxes
  // 3 = lean inviscid state (lean_euler.hpp)
  enum { HALO_MID = 0, HALO_STATE = 1, HALO_QDIR = 2, HALO_LEAN = 3, HALO_LNS = 4 };   // HALO_LNS: lean N-S / mechanism (device)
  int halo_doubles(int group) const;
  void pack_column(int group, int local_i, real* buf) const;
  void unpack_column(int group, int local_i, const real* buf);
  std::function<void(CpuSolver&, int)> halo_exchange;

  // lean inviscid path (off by default on the CPU: the generic stepper is the
  // oracle the device kernels are checked against)
  bool lean = false;
  bool lean_tile = false;   // emulate the device's LDS-tiled lean kernel
  bool lean_sg = true;      // single-gas specialisation when the case allows it
  int lean_tj = 0, lean_cpt = 1;   // tile height override, cells per thread
  int lean_nt = 256;               // threads per emulated tile workgroup (256 / 128 / 64)
  bool lean_sg_ok = false;
  bool lean_ok = false;
  std::string lean_why;
  int lean_state = 0;   // 1: lean arrays authoritative, A/B/F/p stale
  std::vector<real> Spre[2], P2[2];
  std::vector<uint8_t> lb;
  LeanSoA lean_view(bool fromg);
  void lean_materialize();
};

class RefSolver : public SolverBase {
 public:
  explicit RefSolver(Case& cs);
  StepResult do_step(const StepParams& P, bool want_res) override;
  void download(Field&) override {}
  void upload() override {}
  void poison_cell(int gi, int j) override;
  std::vector<CellRecord> core;   // FlowNodeCore2D scratch (NextNode)
};

}  // namespace hf2d
