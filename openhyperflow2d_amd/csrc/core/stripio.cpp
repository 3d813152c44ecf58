#include "stripio.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <sstream>
#include <stdexcept>

#include "checkpoint.hpp"
#include "postproc.hpp"

namespace hf2d {

namespace {

void put(std::string& s, const void* p, size_t n) { s.append((const char*)p, n); }

template <class T>
T get(const std::string& s, size_t& o) {
  T v;
  if (o + sizeof(T) > s.size()) throw std::runtime_error("stripio: short message");
  std::memcpy(&v, s.data() + o, sizeof(T));
  o += sizeof(T);
  return v;
}

void pwrite_all(int fd, const char* p, size_t len, off_t off, const std::string& path) {
  while (len > 0) {
    const ssize_t r = ::pwrite(fd, p, len, off);
    if (r <= 0) throw std::runtime_error("short write to " + path);
    p += r;
    off += r;
    len -= (size_t)r;
  }
}

// column of a cut and whether this rank evaluates it: the owner of the
// column, or rank 0 when the cut lies outside the grid (the integral then
// returns before reading a record)
bool cut_here(const Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, real x0) {
  const int i = (int)(unsigned)(x0 / cs.cfg.dx);
  if (i >= J.nx) return comm.rank() == 0;
  return i >= gi0 && i < gi1;
}

}  // namespace

void strip_exchange_ghosts(Comm& comm, Field& J, int gi0, int gi1) {
  if (comm.size() == 1) return;
  const size_t col = (size_t)J.ny * sizeof(CellRecord);
  std::string m;
  put(m, &gi0, sizeof gi0);
  put(m, &gi1, sizeof gi1);
  put(m, &J.at(gi0, 0), col);
  put(m, &J.at(gi1 - 1, 0), col);
  const std::vector<std::string> all = comm.allgather_bytes(m);
  for (int q = 0; q < (int)all.size(); q++) {
    if (q == comm.rank()) continue;
    size_t o = 0;
    const int a = get<int>(all[q], o), b = get<int>(all[q], o);
    if (all[q].size() != o + 2 * col) throw std::runtime_error("stripio: bad ghost message");
    if (b == gi0 && J.resident(gi0 - 1)) std::memcpy((void*)&J.at(gi0 - 1, 0), all[q].data() + o + col, col);
    if (a == gi1 && J.resident(gi1)) std::memcpy((void*)&J.at(gi1, 0), all[q].data() + o, col);
  }
}

void strip_write_plt(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1,
                     real global_time, bool rewrite) {
  const int ny = cs.cfg.MaxY, r = comm.rank(), n = comm.size();
  const bool last = r == n - 1;
  const GasFlow* cxf = plt_cx_flow(cs);
  // this rank's share of every row (the last rank closes GNUPlot rows)
  std::vector<std::string> rows(ny);
  std::vector<long long> len(ny + 1);
  for (int j = 0; j < ny; j++) {
    std::ostringstream o;
    plt_row(o, cs, J, j, gi0, gi1, cxf);
    if (rewrite && last) o << "\n";
    rows[j] = o.str();
    len[j] = (long long)rows[j].size();
  }
  const std::string head = plt_header(cs, global_time, cs.cfg.MaxX);
  long long base = 0;
  if (r == 0) {
    // rank 0 truncates (rewrite) or finds the end (append) and writes the
    // header before anyone learns the offsets
    int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | (rewrite ? O_TRUNC : 0), 0644);
    if (fd < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    if (!rewrite && ::fstat(fd, &st) == 0) base = (long long)st.st_size;
    try {
      pwrite_all(fd, head.data(), head.size(), (off_t)base, path);
    } catch (...) {
      ::close(fd);
      throw;
    }
    ::close(fd);
  }
  len[ny] = base;
  std::string m((const char*)len.data(), len.size() * sizeof(long long));
  const std::vector<std::string> all = comm.allgather_bytes(m);
  std::vector<const long long*> L(n);
  for (int q = 0; q < n; q++) {
    if (all[q].size() != len.size() * sizeof(long long)) throw std::runtime_error("stripio: bad row lengths");
    L[q] = (const long long*)all[q].data();
  }
  // offset of row j's chunk of rank r: header + the full rows before it +
  // the chunks of the ranks before r in the same row
  long long off = L[0][ny] + (long long)head.size();
  int fd = ::open(path.c_str(), O_WRONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path);
  try {
    for (int j = 0; j < ny; j++) {
      long long mine = off;
      for (int q = 0; q < r; q++) mine += L[q][j];
      if (!rows[j].empty()) pwrite_all(fd, rows[j].data(), rows[j].size(), (off_t)mine, path);
      for (int q = 0; q < n; q++) off += L[q][j];
    }
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
  comm.barrier();   // the file is complete on return, on every rank
}

void strip_write_hf2d(Comm& comm, const std::string& path, const Field& J, int gi0, int gi1) {
  if (comm.rank() == 0) {
    int fd = ::open(path.c_str(), O_WRONLY | O_CREAT, 0644);
    if (fd < 0) throw std::runtime_error("cannot open checkpoint " + path);
    const int rc = ::ftruncate(fd, (off_t)J.nx * J.ny * (off_t)sizeof(CellRecord));
    ::close(fd);
    if (rc != 0) throw std::runtime_error("cannot size checkpoint " + path);
  }
  comm.barrier();
  write_hf2d_slab(path, J, gi0 - J.i0, gi0, gi1 - gi0, J.nx);
  comm.barrier();
}

real strip_pick(Comm& comm, bool have, real v) {
  if (comm.size() == 1) return v;
  std::string m;
  const char h = have ? 1 : 0;
  put(m, &h, 1);
  put(m, &v, sizeof v);
  for (const std::string& s : comm.allgather_bytes(m))
    if (s.size() == 1 + sizeof(real) && s[0]) {
      real x;
      std::memcpy(&x, s.data() + 1, sizeof x);
      return x;
    }
  return 0;
}

std::vector<real> strip_fold(Comm& comm, const std::vector<std::vector<real>>& lists) {
  const size_t k = lists.size();
  std::vector<real> sums(k, 0.);
  if (comm.size() == 1) {
    for (size_t a = 0; a < k; a++) sums[a] = fold_terms(lists[a]);
    return sums;
  }
  std::string m;
  for (const auto& l : lists) {
    const unsigned long long c = l.size();
    put(m, &c, sizeof c);
    put(m, l.data(), l.size() * sizeof(real));
  }
  for (const std::string& s : comm.allgather_bytes(m)) {
    size_t o = 0;
    for (size_t a = 0; a < k; a++) {
      const unsigned long long c = get<unsigned long long>(s, o);
      for (unsigned long long t = 0; t < c; t++) sums[a] += get<real>(s, o);
    }
  }
  return sums;
}

real strip_mass_flow(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, real x0, real y0, real dy) {
  const bool have = cut_here(comm, cs, J, gi0, gi1, x0);
  return strip_pick(comm, have, have ? mass_flow_rate_x(cs, J, x0, y0, dy) : 0.);
}

void strip_cd_cv(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, const GasFlow& f, real out[2]) {
  const Config& C = cs.cfg;
  const bool have = cut_here(comm, cs, J, gi0, gi1, C.x0_nozzle);
  out[0] = strip_pick(comm, have, have ? calc_cd(cs, J, C.x0_nozzle, C.y0_nozzle, C.dy_nozzle, f) : 0.);
  out[1] = strip_pick(comm, have, have ? calc_cv(cs, J, C.x0_nozzle, C.y0_nozzle, C.dy_nozzle, C.p_ambient, f) : 0.);
}

void strip_body_forces(Comm& comm, const Case& cs, const Field& J, int gi0, int gi1, const GasFlow& f, real out[4]) {
  const Config& C = cs.cfg;
  std::vector<std::vector<real>> t(5);
  x_force_terms(cs, J, C.x0_body, C.y0_body, C.dx_body, C.dy_body, gi0, gi1, t[0], t[1]);
  y_force_terms(cs, J, C.x0_body, C.y0_body, C.dx_body, C.dy_body, gi0, gi1, t[2], t[3]);
  wall_span_terms(cs, J, C.x0_body, C.y0_body, C.dx_body, C.dy_body, gi0, gi1, t[4]);
  const std::vector<real> s = strip_fold(comm, t);
  const real fx = s[0] + s[1], fy = s[2] + s[3], pmax = body_pmax(s[4], f);
  out[0] = pmax == 0. ? 0 : fx / pmax;
  out[1] = pmax == 0. ? 0 : fy / pmax;
  out[2] = fx;
  out[3] = fy;
}

void strip_heat_flux_x(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1) {
  const int NX = J.nx;
  std::vector<real> Q(NX, 0.), Al(NX, 0.), Cp(NX, 0.), St(NX, 0.);
  const bool ok = heat_flux_x_cols(cs, J, gi0, gi1, Q.data(), Al.data(), Cp.data(), St.data());
  if (comm.size() > 1) {
    std::string m;
    put(m, &gi0, sizeof gi0);
    put(m, &gi1, sizeof gi1);
    for (const auto* v : {&Q, &Al, &Cp, &St}) put(m, v->data() + gi0, (size_t)(gi1 - gi0) * sizeof(real));
    const std::vector<std::string> all = comm.allgather_bytes(m);
    if (comm.rank() == 0)
      for (const std::string& s : all) {
        size_t o = 0;
        const int a = get<int>(s, o), b = get<int>(s, o);
        for (auto* v : {&Q, &Al, &Cp, &St})
          for (int i = a; i < b; i++) (*v)[i] = get<real>(s, o);
      }
  }
  if (comm.rank() == 0) write_x_heat_flux(path, cs.cfg, ok, Q.data(), Al.data(), Cp.data(), St.data());
}

void strip_heat_flux_y(Comm& comm, const std::string& path, const Case& cs, const Field& J, int gi0, int gi1) {
  std::vector<real> jq;
  heat_flux_y_terms(cs, J, gi0, gi1, jq);
  std::vector<real> Q(J.ny, 0.);
  if (comm.size() == 1) {
    fold_heat_flux_y(Q, jq);
  } else {
    const std::vector<std::string> all =
        comm.allgather_bytes(std::string((const char*)jq.data(), jq.size() * sizeof(real)));
    for (const std::string& s : all) {
      std::vector<real> t(s.size() / sizeof(real));
      if (!t.empty()) std::memcpy(t.data(), s.data(), t.size() * sizeof(real));
      fold_heat_flux_y(Q, t);
    }
  }
  if (comm.rank() == 0) write_y_heat_flux(path, cs.cfg, Q);
}

}  // namespace hf2d
