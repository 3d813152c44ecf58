// DeviceSolver: MI355X backend of the DEEPS time march (see device_solver.hip).
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../core/solver.hpp"

namespace hf2d {

struct LnmArrays;
struct LeanTile;

bool gpu_available();

// In-process stand-in for the RCCL communicator: N DeviceSolvers (one host
// thread each, possibly sharing one GPU) exchange halo buffers with D2D
// copies and reduce scalars on the host.  Same call sites and pack layout as
// the RCCL path; lets the strip decomposition be verified on a single GPU
// (RCCL refuses two ranks on one device).
struct LocalGroup {
  explicit LocalGroup(int n_)
      : n(n_), send_l(n_), send_r(n_), dt_src(n_, nullptr), vals(n_), packs(n_), blobs(n_) {
    const char* j = std::getenv("HF2D_LOCAL_JITTER_US");
    jitter_us = j ? std::max(0, std::atoi(j)) : 0;
  }
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  // race probe (HF2D_LOCAL_JITTER_US = J > 0): every rank sleeps a
  // pseudo-random 0..J us before each barrier, so the threads reach the
  // collectives and the D2D halo copies in varying orders; a result that
  // depends on that order is an ordering hole (tools/strip_outputs_check.py)
  int jitter_us = 0;
  unsigned long long jitter_state = 0x9E3779B97F4A7C15ull;
  void jitter() {
    unsigned long long x;
    {
      std::lock_guard<std::mutex> lk(mu);
      jitter_state ^= jitter_state << 13;
      jitter_state ^= jitter_state >> 7;
      jitter_state ^= jitter_state << 17;
      x = jitter_state;
    }
    std::this_thread::sleep_for(std::chrono::microseconds((long)(x % (unsigned long long)jitter_us)));
  }
  std::vector<real*> send_l, send_r;
  std::vector<const unsigned long long*> dt_src;   // device dt slot of each rank
  std::vector<double> vals;
  std::vector<ResidualPack> packs;
  std::vector<std::string> blobs;   // allgather_bytes slots
  void barrier() {
    if (jitter_us > 0) jitter();
    std::unique_lock<std::mutex> lk(mu);
    const long g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
  double reduce(int rank, double v, int op) {   // 0 min, 1 sum, 2 max
    vals[rank] = v;
    barrier();
    double r = vals[0];
    for (int q = 1; q < n; q++) r = op == 0 ? std::min(r, vals[q]) : op == 1 ? r + vals[q] : std::max(r, vals[q]);
    barrier();
    return r;
  }
};

std::shared_ptr<LocalGroup> make_local_group(int n);

class DeviceSolver : public SolverBase {
 public:
  DeviceSolver(Case& cs, int device = 0, int gi0 = 0, int gi1 = -1);
  ~DeviceSolver() override;
  StepResult do_step(const StepParams& P, bool want_res) override;
  StepResult do_step_eager(const StepParams& P, bool want_res);
  std::pair<int, int> owned_columns() const override { return {gi0, gi1}; }
  void download(Field& J) override;
  void upload() override;
  void cycle_update() override;
  void sync_scalars() override;
  void on_cycle_roll() override;
  void poison_cell(int gi, int j) override;
  void sample_monitors(std::vector<MonitorPoint>& mp) override;
  std::vector<long> probe_idx_host;
  std::vector<real> probe_buf_host;
  void trace_push(const char* name) override;
  void trace_pop() override;
  double time_offset = 0.0, last_dev_time = 0.0;
  void synchronize();
  // ThreadBlockSize = 0: time the lean tile geometries, keep the fastest (before the first step)
  std::string autotune(int steps = 120);
  std::vector<unsigned long long> trace_tile(int steps = 20);
  unsigned long long* tile_trace = nullptr;   // set only inside trace_tile
  void* stream() const;

  // Multi-GPU: RCCL communicator over the strip ranks.
  static std::string nccl_unique_id();
  void init_comm(const std::string& uid, int rank, int nranks);
  // in-process virtual ranks (tests on one GPU; see LocalGroup)
  void init_local(std::shared_ptr<LocalGroup> g, int rank);
  // Multi-GPU: xGMI peer-to-peer mailboxes (hf2d_p2p_xchg).  Every rank
  // exports a descriptor, the descriptors are all-gathered by the caller
  // (torch.distributed, any backend) and imported on every rank; from then on
  // the per-step halo + dt exchange is one device kernel (no RCCL, no host).
  std::string p2p_export(int rank, int nranks);
  void p2p_import(const std::vector<std::string>& descs);
  // timing stand-in: rank `rank` of `nranks` with every peer ready and the
  // neighbours' mailboxes looped back into this rank's own (device_solver.hip)
  void p2p_loopback(int rank, int nranks);
  bool p2p_active() const;
  bool p2p_fuse = false;     // fold the p2p exchange into the lean tile kernel (hf2d_lean_tile_fx)
  bool p2p_queue_check = true;   // p2p_import refuses more in-process ranks than HIP hardware queues allow
  // lean tile dt read (StepParams::dt_read / dt_fold; HF2D_DT_READ): 0 word +
  // shards by scalar loads, 1 by one vector load per lane, 2 the previous
  // step's last workgroup folds them into the word (single GPU)
  int dt_read_mode = 1;
  bool dt_word_valid = false;
  // lean tile: skip stores of beta / CP whose bits did not change (HF2D_SKIP_SAME)
  bool tile_skip_same = false;
  bool fx_step = false, fx_pending = false;
  // fused lean N-S steps: the last step's halo is still in the mailbox; the
  // next fused step's edge tiles unpack it (lns_ghost_prologue, HF2D_GHOST_PROLOGUE)
  bool lns_ghost_pending = false, lns_ghost_prologue = true, lns_last_valid = false, lns_prev_valid = false;
  int lns_pro_uses = 0;
  long lns_prologue_steps = 0;   // fused lean N-S steps that unpacked the previous halo themselves
  const struct ColList* lc_device(const struct ColList& L);
  void p2p_complete(bool keep_lns = false);
  struct FusedX fused_args() const;
  const struct FusedX* fx_device(const struct FusedX& X);
  void p2p_set(bool on);   // off: fall back to RCCL/local; on: only after p2p_import
  int comm_rank() const;
  int comm_size() const;
  void exchange(int group, int dt_slot = -1, void* on_stream = nullptr, bool full = false);
  void exchange_dt(int dt_slot);
  // split-path halos carry only what the next kernels read of a ghost column
  // (halo_fields); false: every field of the group (the A/B of the layouts)
  bool halo_compact = true;
  int ghost_mode = -1;    // SK_* mode the ghost columns were last exchanged for (-1: complete)
  int split_mode() const; // SK_* mode of the split stepper (step_split)
  bool any_cauchy_x = true;   // some node applies d2/dx2 = 0 (reads dS/dx of an x neighbour)
  // RCCL / in-process transports: halo of the edge tiles on a comm stream while
  // the interior tiles compute, then the dt MIN (lean tile steps)
  bool comm_overlap = true;
  // single GPU: the last lean tile step of a host call writes dt / time /
  // the error flag into the pinned host mirror from its own tail, instead of
  // a separate read-back kernel after it (HF2D_HOST_TAIL=0: off)
  bool host_tail = true;
  bool lnm_overlap = false;   // mechanism step: edge tiles first, halo overlapped with the interior (opt-in)
  bool lns_split = false;   // this lean N-S step ran edge-first with its halo overlapped
  bool lnm_split = false;   // this lean mechanism step ran edge-first with its halo overlapped
  bool lns_fx = false;      // this lean N-S step exchanged through the fused mailbox kernel
  long lns_fx_steps = 0;    // lean N-S steps with the fused xGMI mailbox exchange
  long p2p_mwg_exchanges = 0;   // mailbox exchanges through hf2d_p2p_push / hf2d_p2p_unpack
  long overlap_steps = 0;
  // device columns of the fields a halo group carries, in pack order
  void halo_fields(int group, std::vector<real*>& f, bool full = false) const;
  // (o: column offset of each entry, 1 = the second column of a two-column halo)
  void halo_fields(int group, std::vector<real*>& f, std::vector<unsigned char>& o, bool full) const;
  bool ghost_stale = false;   // the ghost columns hold another stepper's representation (refresh before a split step)
  // p2p self-validation (collective over the strip ranks, before the first
  // step): poisons the ghost columns, runs one mailbox exchange of the full
  // state group with a rank-tagged dt, restores the device scalars and
  // returns this rank's checksums of the columns it sent and received and of
  // the folded dt.  p2p_probe_ok checks the all-gathered blobs of every rank.
  std::string p2p_probe();
  std::vector<unsigned long long> fx_trace();   // fused-exchange tail phase clocks (HF2D_FX_SKIP bit 4)
  static bool p2p_probe_ok(const std::vector<std::string>& blobs, int rank, std::string* why);
  void p2p_fallback();   // p2p off, ghost columns refilled over RCCL / the local group

  HostArrays h;           // host staging copy
  int dev = 0;
  int gi0 = 0, gi1 = 0, l_off = 0;
  long nstep = 0;
  int abuf = 0, dsbuf = 0, pbuf = 0, sbuf = 0;  // ping-pong indices (sbuf: current state)
  bool fused = true;      // Euler: single fused predict+fill kernel
  // Inviscid: lean kernel on the reduced state (lean_euler.hpp) when the case
  // is eligible; takes precedence over `fused`.
  bool lean = true;
  bool lean_tile = true;  // LDS-tiled lean kernel for all but the first lean step
  bool lean_plain = false; // flag-free predictor fast path (measured slower: off)
  bool lean_sg = true;     // single-gas specialisation (lean_euler.hpp) if eligible
  int lean_tj = 0;         // tile height override (0: auto, ny split in <= 64)
  int lean_wgcu = 0;       // >0: at most this many tile workgroups resident per CU (LDS request)
  int push_per = 1;        // halo values per thread of the mailbox push kernel (1, 4, 16)
  int lean_occ = 0;        // occupancy target (waves/SIMD) for the hot kernel: 0 or 6 (cpt 1)
  int lean_cpt = 2;        // cells per thread in the tiled kernel: 1 or 2 (2: measured ~20% faster)
  int lean_nt = 256;       // threads per tile workgroup: 256, or 128 / 64 (single gas; small strips)
  int cu_count = 256;
  bool lean_sg_ok = false;
  bool lean_has_cauchy_x = true;   // some node reads dS/dx of an x neighbour (halo must carry it)
  void set_lean_plain(bool on);
  bool lean_ok = false;
  std::string lean_why;
  bool chem_fast = true;  // mechanism mode: compiled-mechanism kinetics kernel when one exists
  bool chem_fast_ok = false;   // the loaded mechanism equals a compiled one
  bool chem_compact = true;    // compiled kinetics over a compacted list of the reacting cells
  // kinetics kernel: 0 auto (compiled VALU kernel if the mechanism has one,
  // else the hiprtc-specialised one, else the MFMA kernel), 1 compiled, 2 MFMA,
  // 3 generic runtime-data VALU, 4 hiprtc-specialised
  int chem_kernel = 0;
  std::string chem_kernel_used;
  // a mechanism without built-in kernels: hiprtc-specialised chem_fast kernels
  // (chem_rtc.hip, compiled at upload, code object cached) instead of the
  // runtime-data MFMA kernel; kernel kind 4
  bool chem_rtc = true;
  bool chem_rtc_ok = false;
  std::string chem_rtc_why;
  bool sgl = true;        // single-gas laminar N-S specialisation (stepkern.hpp fill_cell<SGL>) if eligible
  bool sgl_ok = false;
  int sk_mode = 0;        // SK_GENERIC / SK_SGL / SK_SGT (stepkern.hpp)
  int fill_occ = -1;      // split fill kernels: -1 auto, 0 compiler default, 2/3/4 waves-per-SIMD register budget
  bool split_xcd = true;  // split predict/fill: XCD-aware workgroup order (HF2D_SPLIT_XCD=0 off)
  bool split_xcd_mech = false;   // ... also for the mechanism pair (measured 2 % slower; HF2D_SPLIT_XCD_MECH=1)
  bool mech_lazy = true;  // mechanism N-S fill: species gradients/fluxes inside the heat flux (HF2D_MECH_LAZY=0 off)
  bool grad_every = false; // SGT / mechanism split fill: store the gradients every step, not only on outputs
  std::string sgl_why;
  int lean_state = 0;     // 1: lean arrays authoritative (A/B/F/p stale)
  // Single-gas laminar N-S: one LDS-tiled kernel per step with the fluxes
  // recomputed in the tile (hip/lean_ns.hpp) when eligible (lns_ok: flat,
  // SK_SGL, adiabatic walls, no sources; one strip)
  bool lean_ns = true;
  bool lns_ok = false;
  std::string lns_why;
  int lns_state = 0;      // 1: lean N-S buffers authoritative (committed S, A/B/F, p stale)
  int cbuf = 0;           // lean N-S: CP/mu/lam/k level ping-pong (0: the generic arrays)
  long lns_steps = 0;
  int lns_occ = 0;
  int lns_turb = 2;       // turbulence set of the SGT kernel: 2 k-eps, 3 SST, 4 Spalart-Allmaras
  int lns_prev_mu_t = -1;  // is_mu_t of the previous step (the split fill F_m ran with it)        // 0: compiler register budget; 5 / 6: waves-per-SIMD budget
  void lns_materialize();
  // Mechanism mode (SK_MECH N-S, laminar or k-omega SST): the lean step of
  // hip/lean_mech.hpp (tile kernel + kinetics + reacting-cell state kernel)
  // when eligible (lnm_ok); it shares lns_state / cbuf with the lean N-S path
  bool lean_mech = true;
  bool lnm_ok = false;
  std::string lnm_why;
  int lnm_turb = 0;       // fill_node turbulence set of the kernel: 0 none, 3 SST
  long lnm_steps = 0;
  int lnm_ti = 16;   // mechanism tile columns (16 rows): 16 or 12 (lean_mech.hpp lnm_tile)
  // measurement: per-phase device time of the lean mechanism step (tile
  // kernel, kinetics, reacting-cell state kernel; ms summed) and the number of
  // launches timed (lnm_phase_ms[3]); the host waits for every step's events
  bool lnm_timing = false;
  double lnm_phase_ms[4] = {0, 0, 0, 0};
  // HF2D_STAGGER: staggered start of the inviscid tile kernel's resident
  // dispatch rounds, 10 ns ticks per round of cu_count workgroups; > 0 whole
  // rounds, < 0 a linear ramp (headline 2000x200, 1x MI355X, after the fast
  // divide: off 31.3 us, rounds of 1.5 us 29.9 us; ramp of 0.5 / 1.0 / 1.5 /
  // 2.0 / 3.0 us per round 30.7 / 30.1 / 29.6 / 30.4 / 32.3 us)
  int tile_stagger = -150;
  std::vector<unsigned long long> lnm_trace_fetch();   // HF2D_LNM_TRACE: 12 clocks / ids per workgroup
  std::vector<uint8_t> lean_bytes;
  ScenarioTables scen_host;   // staged for upload (must outlive the async copy)
  void lean_materialize();
  std::unique_ptr<Comm> host_comm;
  // step graphs (see device_solver.hip)
  bool use_graph = true;
  long graph_launches = 0;
  void flush_pending();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl;
  struct GraphCache;
  std::unique_ptr<GraphCache> graph;
  std::vector<StepParams> pending;
  void run_graph();
  uint64_t mode_signature() const;   // kernel-selecting state (graph windows replay only under the same)
  void step_split(const StepParams& P, bool want_res, int slot, int slot_next, int serial, unsigned nblk, bool to_lns);
  bool lns_step_ok(const StepParams& P) const;
  bool lns_entry(const StepParams& P0) const;
  bool lnm_step_ok(const StepParams& P) const;
  void lnm_step(const StepParams& P, bool want_res, int slot, int slot_next, int serial);
  void lnm_launch(const StepParams& P, const LnmArrays& a, const LeanTile& T, bool want_res, int slot, int slot_next,
                  int serial, unsigned ntile);
  // mechanism-mode kinetics of cells [k0, k1) (chem_fast / chem_mech / generic)
  void launch_chem(const StepParams& P, const SoA& mid, const SoA& out, long k0, long k1, unsigned nb, int slot);
};

std::unique_ptr<SolverBase> make_gpu_solver(Case& cs, int device);
std::unique_ptr<SolverBase> make_gpu_strip_solver(Case& cs, int device, int gi0, int gi1, Comm& boot,
                                                  const std::string& transport, std::string& used);

}  // namespace hf2d
