// Strip scatter of a pre-processed Case (the reference's rank-0
// pre-processing and subdomain send, hf2d_start.cpp:143-205): rank 0 builds
// the whole problem once, every rank receives its strip -- the columns it
// owns plus one ghost column each side, and the per-case data (configuration,
// flow lists, wall-node list, eligibility facts of the whole field) -- so no
// other rank ever holds the full 1248 B/cell field or repeats the
// pre-processing.
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "case.hpp"
#include "solver.hpp"

namespace hf2d {

namespace {

constexpr uint64_t STRIP_MAGIC = 0x3150495254534648ull;   // "HFSTRIP1"

struct Writer {
  std::string b;
  template <class T>
  void pod(const T& v) {
    static_assert(std::is_trivially_copyable<T>::value, "POD only");
    b.append((const char*)&v, sizeof v);
  }
  void str(const std::string& s) {
    pod((uint64_t)s.size());
    b += s;
  }
  template <class T>
  void vec(const std::vector<T>& v) {
    static_assert(std::is_trivially_copyable<T>::value, "POD only");
    pod((uint64_t)v.size());
    if (!v.empty()) b.append((const char*)v.data(), v.size() * sizeof(T));
  }
  void table(const Table& t) {
    str(t.name);
    vec(t.x);
    vec(t.y);
  }
};

struct Reader {
  struct View {
    const char* p;
    size_t n;
    size_t size() const { return n; }
    const char* data() const { return p; }
  } b;
  size_t o = 0;
  void need(size_t n) {
    if (o + n > b.size()) throw std::runtime_error("strip blob truncated");
  }
  template <class T>
  void pod(T& v) {
    static_assert(std::is_trivially_copyable<T>::value, "POD only");
    need(sizeof v);
    std::memcpy((void*)&v, b.data() + o, sizeof v);
    o += sizeof v;
  }
  void str(std::string& s) {
    uint64_t n = 0;
    pod(n);
    need(n);
    s.assign(b.data() + o, n);
    o += n;
  }
  template <class T>
  void vec(std::vector<T>& v) {
    uint64_t n = 0;
    pod(n);
    need(n * sizeof(T));
    v.clear();
    v.reserve(n);
    for (uint64_t k = 0; k < n; k++) {   // (no default constructor needed: GasFlow)
      typename std::aligned_storage<sizeof(T), alignof(T)>::type tmp;
      std::memcpy((void*)&tmp, b.data() + o + k * sizeof(T), sizeof(T));
      v.push_back(*reinterpret_cast<const T*>(&tmp));
    }
    o += n * sizeof(T);
  }
  void table(Table& t) {
    str(t.name);
    vec(t.x);
    vec(t.y);
  }
};

// Every Config member, in declaration order (case.hpp); a member added there
// must be added here (the strip tests compare strip runs with one rank byte
// for byte).
template <class IO, class C>
void config_io(IO& io, C& c) {
  io.str(c.project);
  io.str(c.out_file);
  io.str(c.err_file);
  io.str(c.swap_file);
  io.str(c.tecplot_file);
  io.pod(c.isVerboseOutput);
  io.pod(c.bff);
  io.pod(c.MaxX);
  io.pod(c.MaxY);
  io.pod(c.dx);
  io.pod(c.dy);
  io.pod(c.SigW);
  io.pod(c.SigF);
  io.pod(c.delta_bl);
  io.pod(c.TurbMod);
  io.pod(c.TurbStartIter);
  io.pod(c.TurbExtModel);
  io.pod(c.isTurbulenceReset);
  io.pod(c.FT);
  io.pod(c.ProblemType);
  io.pod(c.CFL);
  io.pod(c.ViscousCFL);
  io.pod(c.SSTWallDistance);
  io.pod(c.LaggedDt);
  io.pod(c.WallBlendCells);
  io.pod(c.WallBlendFactor);
  io.pod(c.ThreadBlockSize);
  io.table(c.CFL_Scenario);
  io.table(c.beta_Scenario);
  io.pod(c.NSaveStep);
  io.pod(c.Nmax);
  io.pod(c.NOutStep);
  io.pod(c.isAlternateRMS);
  io.pod(c.isIgnoreUnsetNodes);
  io.pod(c.MonitorIndex);
  io.pod(c.ExitMonitorValue);
  io.vec(c.monitors);
  io.pod(c.beta0);
  io.pod(c.nrbc_beta0);
  io.pod(c.species);
  io.pod(c.isAdiabaticWall);
  io.pod(c.Hu);
  io.pod(c.Ts0);
  io.pod(c.isOutHeatFluxX);
  io.pod(c.Cp_Flow_index);
  io.pod(c.y_max);
  io.pod(c.y_min);
  io.pod(c.isOutHeatFluxY);
  io.pod(c.is_p_asterisk_out);
  io.pod(c.is_Cx_calc);
  io.pod(c.Cx_Flow_index);
  io.pod(c.x0_body);
  io.pod(c.y0_body);
  io.pod(c.dx_body);
  io.pod(c.dy_body);
  io.pod(c.is_Cd_calc);
  io.pod(c.Cd_Flow_index);
  io.pod(c.x0_nozzle);
  io.pod(c.y0_nozzle);
  io.pod(c.dy_nozzle);
  io.pod(c.p_ambient);
  io.pod(c.InitTime);
  io.vec(c.xcuts);
  io.vec(c.sources);
  io.pod(c.semantics);
  io.pod(c.chem_model);
  io.str(c.mechanism);
  io.pod(c.chem_nsub);
  io.pod(c.chem_tmin);
}

std::vector<int> pairs_flat(const std::vector<std::pair<int, int>>& v) {
  std::vector<int> f;
  f.reserve(2 * v.size());
  for (const auto& p : v) {
    f.push_back(p.first);
    f.push_back(p.second);
  }
  return f;
}
std::vector<std::pair<int, int>> pairs_of(const std::vector<int>& f) {
  std::vector<std::pair<int, int>> v(f.size() / 2);
  for (size_t k = 0; k < v.size(); k++) v[k] = {f[2 * k], f[2 * k + 1]};
  return v;
}

}  // namespace

void Case::compute_facts() {
  if (!J.whole()) throw std::runtime_error("Case::compute_facts needs the whole field");
  merge_facts({facts_part()});
}

std::string Case::pack_strip_header(int a, int b) const {
  if (!J.whole()) throw std::runtime_error("Case::pack_strip: this Case holds a strip only");
  if (a < 0 || b > J.nx || a >= b) throw std::runtime_error("Case::pack_strip: bad column range");
  Case& self = const_cast<Case&>(*this);
  if (!facts.valid) self.compute_facts();
  Writer w;
  w.pod(STRIP_MAGIC);
  w.pod((uint32_t)sizeof(CellRecord));
  config_io(w, self.cfg);
  w.pod((int)(cfg.mech != nullptr));
  if (cfg.mech) {
    w.str(cfg.mech->name);
    w.str(cfg.mech->source);
    w.pod((uint64_t)cfg.mech->species.size());
    for (const auto& s : cfg.mech->species) w.str(s);
    w.pod(cfg.mech->data);
  }
  w.vec(flows);
  w.vec(flows2d);
  w.vec(pairs_flat(wall_nodes));
  w.vec(wall_dirs);
  w.vec(wall_rays);
  w.vec(pairs_flat(subdomains));
  w.pod(dt0);
  w.pod(global_time);
  w.pod(preloaded);
  w.pod(restart_iter);
  w.str(swap_path);
  // facts of the whole field
  w.pod(facts.lean_ok);
  w.str(facts.lean_why);
  w.pod(facts.sk_mode);
  w.str(facts.sk_why);
  w.pod(facts.single_gas);
  w.pod(facts.any_cauchy_x);
  w.pod(facts.species_cauchy);
  // the strip's shape; its payload (records, then species) follows
  w.pod(J.nx);
  w.pod(J.ny);
  w.pod(a);
  w.pod(b);
  const int ns = mech_rhoY.empty() ? 0 : (int)(mech_rhoY.size() / (size_t)mech_n());
  w.pod(ns);
  return w.b;
}

size_t Case::strip_payload_bytes(int a, int b) const {
  const size_t per = (size_t)(b - a) * J.ny;
  const int ns = mech_rhoY.empty() ? 0 : (int)(mech_rhoY.size() / (size_t)mech_n());
  return per * sizeof(CellRecord) + (size_t)ns * per * sizeof(real);
}

void Case::read_strip_payload(int a, int b, size_t off, char* dst, size_t n) const {
  const size_t per = (size_t)(b - a) * J.ny, rec = per * sizeof(CellRecord);
  if (off + n > strip_payload_bytes(a, b)) throw std::runtime_error("read_strip_payload: out of range");
  while (n) {
    size_t k;
    if (off < rec) {   // records of columns [a, b) are contiguous
      k = std::min(n, rec - off);
      std::memcpy(dst, (const char*)&J.at(a, 0) + off, k);
    } else {           // species s, columns [a, b): contiguous per species
      const size_t so = off - rec, sp = so / (per * sizeof(real)), in = so % (per * sizeof(real));
      k = std::min(n, per * sizeof(real) - in);
      std::memcpy(dst, (const char*)&mech_rhoY[mech_idx((int)sp, a, 0)] + in, k);
    }
    dst += k;
    off += k;
    n -= k;
  }
}

std::string Case::pack_strip(int a, int b) const {
  a = std::max(a, 0);
  b = std::min(b, J.nx);
  std::string blob = pack_strip_header(a, b);
  const size_t h = blob.size(), n = strip_payload_bytes(a, b);
  blob.resize(h + n);
  read_strip_payload(a, b, 0, &blob[h], n);
  return blob;
}

Case Case::unpack_strip_header(const char* data, size_t size, std::ostream* log, size_t* used) {
  Reader r{{data, size}};
  uint64_t magic = 0;
  uint32_t rec = 0;
  r.pod(magic);
  r.pod(rec);
  if (magic != STRIP_MAGIC || rec != sizeof(CellRecord)) throw std::runtime_error("not a strip blob of this build");
  Case cs;
  cs.log = log;
  config_io(r, cs.cfg);
  int has_mech = 0;
  r.pod(has_mech);
  if (has_mech) {
    auto m = std::make_shared<MechInfo>();
    r.str(m->name);
    r.str(m->source);
    uint64_t n = 0;
    r.pod(n);
    m->species.resize(n);
    for (auto& s : m->species) r.str(s);
    r.pod(m->data);
    cs.cfg.mech = m;
  }
  r.vec(cs.flows);
  r.vec(cs.flows2d);
  std::vector<int> flat;
  r.vec(flat);
  cs.wall_nodes = pairs_of(flat);
  r.vec(cs.wall_dirs);
  r.vec(cs.wall_rays);
  r.vec(flat);
  cs.subdomains = pairs_of(flat);
  r.pod(cs.dt0);
  r.pod(cs.global_time);
  r.pod(cs.preloaded);
  r.pod(cs.restart_iter);
  r.str(cs.swap_path);
  r.pod(cs.facts.lean_ok);
  r.str(cs.facts.lean_why);
  r.pod(cs.facts.sk_mode);
  r.str(cs.facts.sk_why);
  r.pod(cs.facts.single_gas);
  r.pod(cs.facts.any_cauchy_x);
  r.pod(cs.facts.species_cauchy);
  cs.facts.valid = true;
  int nx = 0, ny = 0, a = 0, b = 0, ns = 0;
  r.pod(nx);
  r.pod(ny);
  r.pod(a);
  r.pod(b);
  r.pod(ns);
  cs.J.nx = nx;
  cs.J.ny = ny;
  cs.J.i0 = a;
  cs.J.nxl = b - a;
  const size_t per = (size_t)(b - a) * ny;
  cs.J.c.resize(per);
  cs.mech_rhoY.assign((size_t)ns * per, 0.0);
  if (used) *used = r.o;
  return cs;
}

void Case::write_strip_payload(size_t off, const char* src, size_t n) {
  const size_t per = (size_t)J.nxl * J.ny, rec = per * sizeof(CellRecord);
  if (off + n > rec + mech_rhoY.size() * sizeof(real)) throw std::runtime_error("write_strip_payload: out of range");
  const size_t k = off < rec ? std::min(n, rec - off) : 0;
  if (k) std::memcpy((char*)J.c.data() + off, src, k);
  if (n > k) std::memcpy((char*)mech_rhoY.data() + (off + k - rec), src + k, n - k);
}

Case Case::unpack_strip(const std::string& blob, std::ostream* log) { return unpack_strip(blob.data(), blob.size(), log); }

Case Case::unpack_strip(const char* data, size_t size, std::ostream* log) {
  size_t used = 0;
  Case cs = unpack_strip_header(data, size, log, &used);
  const size_t n = cs.J.c.size() * sizeof(CellRecord) + cs.mech_rhoY.size() * sizeof(real);
  if (used + n != size) throw std::runtime_error("strip blob size mismatch");
  cs.write_strip_payload(0, data + used, n);
  return cs;
}

}  // namespace hf2d
