#include "checkpoint.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <algorithm>
#include <stdexcept>
#include <fstream>
#include <sstream>

namespace hf2d {

namespace {
bool pread_all(int fd, void* buf, size_t len, off_t off) {
  char* p = (char*)buf;
  const size_t chunk = 1UL << 30;
  while (len > 0) {
    ssize_t r = ::pread(fd, p, std::min(len, chunk), off);
    if (r <= 0) return false;
    p += r;
    off += r;
    len -= (size_t)r;
  }
  return true;
}
bool pwrite_all(int fd, const void* buf, size_t len, off_t off) {
  const char* p = (const char*)buf;
  const size_t chunk = 1UL << 30;
  while (len > 0) {
    ssize_t r = ::pwrite(fd, p, std::min(len, chunk), off);
    if (r <= 0) return false;
    p += r;
    off += r;
    len -= (size_t)r;
  }
  return true;
}
}  // namespace

bool read_hf2d(const std::string& path, Field& J) {
  if (!J.whole()) throw std::runtime_error("read_hf2d: the field holds a strip only (use the per-rank slab reader)");
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return false;
  const size_t want = (size_t)J.nx * J.ny * sizeof(CellRecord);
  if ((size_t)st.st_size != want) return false;
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  bool ok = pread_all(fd, J.c.data(), want, 0);
  ::close(fd);
  return ok;
}

bool read_hf2d_window(const std::string& path, Field& J) {
  if (!J.windowed()) throw std::runtime_error("read_hf2d_window: not a windowed field");
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return false;
  const size_t rec = sizeof(CellRecord), want = (size_t)J.nx * J.ny * rec;
  if ((size_t)st.st_size != want) return false;
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  // the rank's own slab: contiguous x-major columns [i0, i0 + nxl)
  bool ok = J.c.empty() || pread_all(fd, J.c.data(), J.c.size() * rec, (off_t)((size_t)J.i0 * J.ny * rec));
  // the flag words of every other column, streamed in ~8 MB blocks of whole columns
  const int per = std::max(1, (int)((8u << 20) / (rec * (size_t)J.ny)));
  std::vector<CellRecord> blk;
  for (int a = 0; ok && a < J.nx; a += per) {
    const int b = std::min(J.nx, a + per);
    if (a >= J.i0 && b <= J.i0 + J.nxl) continue;
    blk.resize((size_t)(b - a) * J.ny);
    ok = pread_all(fd, blk.data(), blk.size() * rec, (off_t)((size_t)a * J.ny * rec));
    for (int i = a; ok && i < b; i++) {
      if (J.resident(i)) continue;
      for (int j = 0; j < J.ny; j++) {
        const CellRecord& c = blk[(size_t)(i - a) * J.ny + j];
        J.g[(size_t)i * J.ny + j] = CellFlags{c.CT, c.TurbType};
      }
    }
  }
  ::close(fd);
  return ok;
}

bool read_hf2d_record(const std::string& path, int nx, int ny, int i, int j, CellRecord& out) {
  if (!checkpoint_image_present(path, nx, ny)) return false;
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  const bool ok = pread_all(fd, &out, sizeof(CellRecord), (off_t)(((size_t)i * ny + j) * sizeof(CellRecord)));
  ::close(fd);
  return ok;
}

void write_hf2d(const std::string& path, const Field& J) {
  if (!J.whole()) throw std::runtime_error("write_hf2d: the field holds a strip only (use write_hf2d_slab)");
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT, 0644);
  if (fd < 0) throw std::runtime_error("cannot open checkpoint " + path);
  const size_t len = (size_t)J.nx * J.ny * sizeof(CellRecord);
  bool ok = pwrite_all(fd, J.c.data(), len, 0);
  if (ok) ok = ::ftruncate(fd, (off_t)len) == 0;
  ::close(fd);
  if (!ok) throw std::runtime_error("short write to checkpoint " + path);
}

bool checkpoint_image_present(const std::string& path, int nx, int ny) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 && (size_t)st.st_size == (size_t)nx * ny * sizeof(CellRecord);
}

void create_zero_hf2d(const std::string& path, int nx, int ny) {
  const off_t len = (off_t)nx * ny * (off_t)sizeof(CellRecord);
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("cannot create checkpoint " + path);
  const int rc = ::ftruncate(fd, len);
  ::close(fd);
  if (rc != 0) throw std::runtime_error("cannot size checkpoint " + path);
}

void write_hf2d_slab(const std::string& path, const Field& local, int local_i0, int global_i0, int ncols,
                     int global_nx) {
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT, 0644);
  if (fd < 0) throw std::runtime_error("cannot open checkpoint " + path);
  const size_t col = (size_t)local.ny * sizeof(CellRecord);
  bool ok = pwrite_all(fd, &local.c[(size_t)local_i0 * local.ny], col * ncols, (off_t)(col * global_i0));
  (void)global_nx;
  ::close(fd);
  if (!ok) throw std::runtime_error("short write to checkpoint " + path);
}

void write_meta(const std::string& path, long iteration, double dt, double time) {
  std::ofstream f(path + ".meta");
  char b[256];
  std::snprintf(b, sizeof b, "{\"format\": \"hf2d-v1\", \"record_bytes\": 1248, \"iteration\": %ld, \"dt\": %.17g, \"time\": %.17g}\n",
                iteration, dt, time);
  f << b;
}

bool read_meta(const std::string& path, long& iteration, double& dt, double& time) {
  std::ifstream f(path + ".meta");
  if (!f.is_open()) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  auto num = [&](const char* key, double& out) {
    size_t p = s.find(key);
    if (p == std::string::npos) return false;
    p = s.find(':', p);
    if (p == std::string::npos) return false;
    out = std::atof(s.c_str() + p + 1);
    return true;
  };
  double it = 0;
  if (!num("\"iteration\"", it) || !num("\"dt\"", dt) || !num("\"time\"", time)) return false;
  iteration = (long)it;
  return true;
}

}  // namespace hf2d
