// Problem definition: solver configuration read from the deck plus the
// pre-processed cell field (host AoS records in x-major order).
//
// Reference correspondence:
//   Config::load        InitSharedData (libDEEPS2D/deeps2d_core.cpp:160-499)
//   Case::preprocess    InitDEEPS2D (deeps2d_core.cpp:2835-4682) + the serial
//                       N-S tail of main() (hf2d_start.cpp:292-303)
#pragma once

#include <functional>
#include <memory>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"
#include "deck.hpp"
#include "gasdyn.hpp"
#include "physics.hpp"
#include "mechanism_io.hpp"

namespace hf2d {

struct MonitorPoint {
  real x = 0, y = 0;
  real p = 0, T = 0;
};

struct XCut {
  real x0 = 0, y0 = 0, dy = 0;
};

struct GasSource {
  int sx, sy, ex, ey, comp;
  real Cp, Ms, T, Tf;
  int start_iter;
};

enum class Semantics { MPI = 0, SERIAL = 1 };

// (scalars in double in every build: the FP32 build keeps the deck's geometry
// and parameters in double and rounds only the flow state)
struct Config {
  // files
  std::string project, out_file, err_file, swap_file, tecplot_file;
  // globals
  int isVerboseOutput = 0, bff = 0;
  int MaxX = 0, MaxY = 0;
  double dx = 0, dy = 0;
  double SigW = 0, SigF = 0, delta_bl = 0;
  int TurbMod = 0, TurbStartIter = 0, TurbExtModel = 0, isTurbulenceReset = 0;
  int FT = FT_FLAT, ProblemType = SM_EULER;
  double CFL = 0;
  // new key (not in the reference): viscous time-step bound for N-S,
  // dt <= ViscousCFL * rho / ((mu + mu_t) (1/dx^2 + 1/dy^2)); 0 = off (reference)
  double ViscousCFL = 0;
  // new key: k-omega SST wall omega = 60 nu / (beta1 d1^2) with d1 = SSTWallDistance *
  // min(dx, dy): 1.0 (default) is Menter's distance of the first cell off the wall node
  double SSTWallDistance = 1.0;
  // new key: lagged time step.  0 (default, the reference):
  // step n+1 uses dt = MIN over every rank's cells of the local dt of step n.
  // 1: step n+1 uses the MIN of step n-1, so a strip only waits for its two
  // neighbours' halos before its next step and the all-rank MIN has a whole
  // step to arrive (the first two steps use the initial dt).
  int LaggedDt = 0;
  // new key: near-wall blend (0 = off, the reference).  N > 0: in the first N
  // cells off a no-slip wall the DEEPS blend of the TANGENTIAL momentum leaves
  // out the wall-normal neighbours (the blend's (1 - beta) dyy/2 dy^2/dt
  // diffusion across the viscous sublayer carries part of the wall stress
  // otherwise; profiles/flat_plate_validation.md).  The streamwise blend,
  // and every other equation's, are unchanged.
  int WallBlendCells = 0;
  // ... keeping this fraction of the wall-normal neighbours' weight (0: none;
  // removing it altogether leaves the wide-stencil viscous term without
  // odd-even damping: the SST plate went unstable within 2000 steps)
  double WallBlendFactor = 0.0;
  // UG item 162 (CUDA in the reference): 0 = auto-calibrate the kernel
  // geometry on the device (DeviceSolver::autotune), > 0 = fixed heuristic
  int ThreadBlockSize = 0;
  Table CFL_Scenario, beta_Scenario;
  int NSaveStep = 1, Nmax = 1, NOutStep = 1;
  int isAlternateRMS = 0, isIgnoreUnsetNodes = 0, MonitorIndex = 0;
  double ExitMonitorValue = 0;
  std::vector<MonitorPoint> monitors;
  double beta0 = 0, nrbc_beta0 = 0;
  SpeciesProps species;
  int isAdiabaticWall = 1;
  double Hu[NSPEC] = {0, 0, 0, 0};
  // pre-processor
  double Ts0 = 0;
  int isOutHeatFluxX = 0, Cp_Flow_index = 0, y_max = 0, y_min = 0, isOutHeatFluxY = 0;
  int is_p_asterisk_out = 0;
  int is_Cx_calc = 0, Cx_Flow_index = 0;
  double x0_body = 0, y0_body = 0, dx_body = 0, dy_body = 0;
  int is_Cd_calc = 0, Cd_Flow_index = 0;
  double x0_nozzle = 0, y0_nozzle = 0, dy_nozzle = 0, p_ambient = 0;
  double InitTime = 0;
  std::vector<XCut> xcuts;
  std::vector<GasSource> sources;
  // runtime options (not in decks; defaults reproduce the reference MPI build)
  Semantics semantics = Semantics::MPI;
  int chem_model = CRM_ZELDOVICH;
  // detailed finite-rate chemistry (new keys): ChemicalReactionsModel = 2 and
  // Mechanism = <built-in name | file.mech> select mechanism mode; the
  // ChemSubsteps point-implicit substeps run per flow step in every cell
  // hotter than ChemTmin [K]
  std::string mechanism;
  std::shared_ptr<MechInfo> mech;
  int chem_nsub = 1;
  double chem_tmin = 300.0;
  bool mech_mode() const { return chem_model == CRM_ARRENIUS && mech != nullptr; }
  int mech_ns() const { return mech ? mech->data.ns : 0; }

  void load_globals(InputDeck& d);   // InitSharedData
  FillParams fill_params() const;    // static FlowNode2D parameters
  int num_active_eq() const;         // max equations used by any cell model
};

// Cell field on the host: x-major (idx = i*MaxY + j) like the .hf2d file.
// A strip rank keeps only the columns [i0, i0 + nxl) resident (its strip plus
// one ghost column each side, Field::trim); nx stays the global width and
// at() takes global column indices.
//
// Windowed pre-processing (Case::from_deck_window): a strip rank builds the
// records of its resident columns only, while the geometry steps -- bounds,
// contours, flood fills, wall / NRBC tagging -- run over the whole grid on a
// 16 B/cell plane of the two flag words (CT, TurbType) of the non-resident
// cells.  ct() / tt() / is() address either, so every geometry step sees the
// whole grid's flags and every state write lands only in resident records.
struct CellFlags {
  u64 CT = 0, TurbType = 0;
};
struct Field {
  int nx = 0, ny = 0;
  int i0 = 0, nxl = 0;   // resident columns
  std::vector<CellRecord> c;
  std::vector<CellFlags> g;   // windowed pre-processing: flags of every cell (empty otherwise)
  void resize(int X, int Y);
  // records of the columns [a, b) only, plus the whole grid's flag plane
  void resize_window(int X, int Y, int a, int b);
  CellRecord& at(int i, int j) { return c[(size_t)(i - i0) * ny + j]; }
  const CellRecord& at(int i, int j) const { return c[(size_t)(i - i0) * ny + j]; }
  bool in(long i, long j) const { return i >= 0 && j >= 0 && i < nx && j < ny; }
  bool resident(long i) const { return i >= i0 && i < i0 + nxl; }
  bool whole() const { return i0 == 0 && nxl == nx; }
  bool windowed() const { return !g.empty(); }
  u64& ct(int i, int j) { return resident(i) ? at(i, j).CT : g[(size_t)i * ny + j].CT; }
  u64 ct(int i, int j) const { return resident(i) ? at(i, j).CT : g[(size_t)i * ny + j].CT; }
  u64& tt(int i, int j) { return resident(i) ? at(i, j).TurbType : g[(size_t)i * ny + j].TurbType; }
  u64 tt(int i, int j) const { return resident(i) ? at(i, j).TurbType : g[(size_t)i * ny + j].TurbType; }
  bool is(int i, int j, u64 mask) const { return (ct(i, j) & mask) == mask; }
  void drop_flags() { std::vector<CellFlags>().swap(g); }
  // drop every column outside [a, b) (global indices, clipped to the grid)
  void trim(int a, int b);
};

// [gi0, gi1) per rank with about equal active (non-solid) cells per strip:
// the same cut as parallel/strips.py balanced_columns (flags only: works on
// a windowed field's flag plane)
std::vector<std::pair<int, int>> balanced_columns(const Field& J, int nparts);

// Whole-field eligibility of the specialised steppers (lean.cpp), evaluated
// on the full pre-processed field: a strip rank that never held it
// (Case::unpack_strip) uses these, so every rank takes the same kernel path.
struct CaseFacts {
  bool valid = false;
  bool lean_ok = false;
  std::string lean_why;
  int sk_mode = 0;
  std::string sk_why;
  bool single_gas = false, any_cauchy_x = false, species_cauchy = false;
};
// The cell-level part of the facts over the resident records of one strip
// (lean.cpp facts_part); facts_merge folds the parts of all strips, in rank
// (= column) order, with the deck-level conditions into the whole field's
// facts -- the same answer, reasons included, as one pass over the whole field.
struct FactsPart {
  bool single_gas = true, any_cauchy_x = false, species_cauchy = false;
  bool lean_cells_ok = true;   // first failing cell's reason otherwise
  std::string lean_why;
  bool sk_cells_ok = true;
  std::string sk_why;
  bool laminar = true;
  std::string pack() const;
  static FactsPart unpack(const std::string& b);
};

class Case {
 public:
  Config cfg;
  Field J;
  std::vector<GasFlow> flows, flows2d;
  std::vector<std::pair<int, int>> wall_nodes;     // (i, j)
  // per wall node: directions into the flow (WD_* bits: the neighbour there
  // is gas, the opposite one a solid cell or the lower / upper grid edge); WallBlendCells
  std::vector<uint8_t> wall_dirs;
  // WallBlendCells: per wall node and direction (x+, x-, y+, y-) the number of
  // cells the blend covers -- the ray stops at the first solid cell or the
  // grid edge.  Measured on the whole grid (collect_wall_nodes), so every
  // strip of a decomposition flags the same cells.
  std::vector<uint8_t> wall_rays;
  std::vector<std::pair<int, int>> subdomains;     // ScanArea [start, end) pairs
  real dt0 = 1.0;
  real global_time = 0.0;
  bool preloaded = false;
  long restart_iter = 0;     // iteration count from the .hf2d.meta sidecar of a preloaded checkpoint
  std::string swap_path;     // resolved checkpoint path ("" = none)
  std::ostream* log = nullptr;
  // mechanism mode: species partial densities, species-major
  // [ns][resident columns * MaxY] (the same columns as J)
  std::vector<real> mech_rhoY;
  std::string species_path() const { return swap_path + ".species"; }
  long mech_n() const { return (long)J.nxl * J.ny; }
  size_t mech_idx(int sp, int gi, int j) const { return (size_t)sp * mech_n() + (size_t)(gi - J.i0) * J.ny + j; }
  // Strip ranks: keep only the columns [a, b) of J and mech_rhoY resident
  // (after the backend uploaded its strip; host RSS then scales with the strip)
  void trim_to_columns(int a, int b);
  CaseFacts facts;

  // Strip scatter (case_io.cpp; the reference pre-processes on rank 0 and
  // sends each rank its subdomain, hf2d_start.cpp:143-205): the per-case data
  // and the columns [a, b) of a whole Case as bytes, and the strip Case of
  // such a blob (columns [a, b) resident, facts of the whole field).
  void compute_facts();
  std::string pack_strip(int a, int b) const;
  static Case unpack_strip(const std::string& blob, std::ostream* log = nullptr);
  static Case unpack_strip(const char* data, size_t size, std::ostream* log = nullptr);
  // the same in pieces (the payload -- records, then species -- sent in
  // chunks straight into the receiving Case: no whole-strip buffer)
  std::string pack_strip_header(int a, int b) const;
  size_t strip_payload_bytes(int a, int b) const;
  void read_strip_payload(int a, int b, size_t off, char* dst, size_t n) const;
  static Case unpack_strip_header(const char* data, size_t size, std::ostream* log = nullptr, size_t* used = nullptr);
  void write_strip_payload(size_t off, const char* src, size_t n);

  // Build the whole problem from a deck.  workdir is where <Project>.hf2d is
  // looked up; checkpoint=false ignores any existing swap file.
  static Case from_deck(InputDeck deck, const std::string& workdir = ".", bool use_checkpoint = true,
                        std::ostream* log = nullptr);
  // Strip-local pre-processing (no whole-field copy anywhere):
  // the same pre-processor with records for the columns [a, b) only and the
  // whole grid's flags in a 16 B/cell plane; a checkpoint restart reads the
  // rank's own slab of the .hf2d (plus the flag words of the rest).  The
  // facts are not valid until merge_facts() got every strip's facts_part().
  static Case from_deck_window(InputDeck deck, const std::string& workdir, bool use_checkpoint, int a, int b,
                               std::ostream* log = nullptr);
  // The active-cell-balanced strips of a deck from a flags-only pass (no
  // records at all): what every rank computes before its windowed pass.
  static std::vector<std::pair<int, int>> partition_deck(InputDeck deck, const std::string& workdir,
                                                         bool use_checkpoint, int nparts);
  FactsPart facts_part() const;
  void merge_facts(const std::vector<FactsPart>& parts);
  CaseFacts fold_facts(const std::vector<FactsPart>& parts) const;   // (merge_facts without storing)

  // Individual pre-processing steps (public for tests).
  void fill_node(CellRecord& n, int is_mu_t, int is_init) const;
  void set_wall_nodes();
  void collect_wall_nodes();
  void set_min_distance_to_wall(real x0 = 0.0);
  // the reference's O(cells x walls) scan (oracle for the bucketed search)
  void set_min_distance_to_wall_bruteforce(real x0 = 0.0);
  void recalc_y_plus();
  void set_init_boundary_layer(real delta);
  int set_non_reflected_bc();
  void scan_area(int num_parts);
  void set_sources(int iter = 0);
  std::vector<std::pair<int, int>> partition_columns(int num_parts) const;
  // mechanism mode: slot -> species split of the pre-processed field, and the
  // matching record state (rho from p and T, thermally perfect rho*E)
  void init_mechanism(std::vector<real>& rhoY) const;
  void apply_mechanism_state(const std::vector<real>& rhoY);
  void refresh_mechanism_primitives();

 private:
  int win_a = -1, win_b = -1;   // windowed pre-processing: resident columns (-1: the whole grid)
  // record (i, j) as the geometry steps left it: resident, or read from the
  // preloaded checkpoint (windowed restart), or nullptr
  const CellRecord* far_record(int i, int j);
  struct FarRec {
    long key;
    CellRecord r;
    bool reset;   // scan_area's turbulence reset applied
  };
  std::vector<FarRec> far_cache;
  bool far_turb_reset = false;   // scan_area reset the turbulence state: far records get it too
  void turb_reset_record(CellRecord& n, u64 tt) const;
  void load_and_preprocess(InputDeck& deck, const std::string& workdir, bool use_checkpoint, bool flags_only = false);
  void preprocess(InputDeck& d, const std::string& workdir, bool use_checkpoint);
};

}  // namespace hf2d
