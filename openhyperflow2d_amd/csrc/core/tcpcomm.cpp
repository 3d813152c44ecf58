#include "tcpcomm.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace hf2d {

namespace {

[[noreturn]] void fail(const std::string& what) {
  throw std::runtime_error("TcpComm: " + what + " (" + std::strerror(errno) + ")");
}

void send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) fail("send");
    c += k;
    n -= (size_t)k;
  }
}

void recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k == 0) throw std::runtime_error("TcpComm: peer closed the connection (a rank exited)");
    if (k < 0) fail("recv");
    c += k;
    n -= (size_t)k;
  }
}

void send_blob(int fd, const std::string& s) {
  const unsigned long long n = s.size();
  send_all(fd, &n, sizeof n);
  if (n) send_all(fd, s.data(), s.size());
}

std::string recv_blob(int fd) {
  unsigned long long n = 0;
  recv_all(fd, &n, sizeof n);
  std::string s(n, '\0');
  if (n) recv_all(fd, &s[0], n);
  return s;
}

void tune(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

int listen_on(const std::string& addr, int port, int backlog, int* bound_port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) fail("socket");
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (::inet_pton(AF_INET, addr.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(fd, (sockaddr*)&a, sizeof a) != 0) {
    ::close(fd);
    fail("bind " + addr + ":" + std::to_string(port));
  }
  if (::listen(fd, backlog) != 0) {
    ::close(fd);
    fail("listen");
  }
  if (bound_port) {
    socklen_t l = sizeof a;
    ::getsockname(fd, (sockaddr*)&a, &l);
    *bound_port = ntohs(a.sin_port);
  }
  return fd;
}

// poll() that survives signals: SIGINT/SIGTERM handlers (installed without
// SA_RESTART so the solver can checkpoint) interrupt it with EINTR; retry with
// the remaining time.  Returns poll's result (0 = timed out).
int poll_retry(pollfd* p, int np, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const double left = timeout_s - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const int rc = ::poll(p, np, left > 0 ? (int)(left * 1000) : 0);
    if (rc >= 0 || errno != EINTR) return rc;
  }
}

int accept_one(int lfd, double timeout_s, uint32_t* peer_addr = nullptr) {
  pollfd p{lfd, POLLIN, 0};
  const int rc = poll_retry(&p, 1, timeout_s);
  if (rc <= 0) fail("timed out waiting for a peer to connect");
  sockaddr_in a{};
  socklen_t l = sizeof a;
  int fd;
  do fd = ::accept(lfd, (sockaddr*)&a, &l);
  while (fd < 0 && errno == EINTR);
  if (fd < 0) fail("accept");
  if (peer_addr) *peer_addr = a.sin_addr.s_addr;
  tune(fd);
  return fd;
}

int connect_retry(sockaddr_in a, const std::string& addr, double timeout_s);

int connect_retry(const std::string& addr, int port, double timeout_s) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (::inet_pton(AF_INET, addr.c_str(), &a.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (::getaddrinfo(addr.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw std::runtime_error("TcpComm: cannot resolve " + addr);
    a.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
    ::freeaddrinfo(res);
  }
  return connect_retry(a, addr, timeout_s);
}

int connect_retry(sockaddr_in a, const std::string& addr, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) fail("socket");
    if (::connect(fd, (sockaddr*)&a, sizeof a) == 0) {
      tune(fd);
      return fd;
    }
    ::close(fd);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      fail("cannot connect to " + addr + ":" + std::to_string(ntohs(a.sin_port)));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace

TcpComm::TcpComm(int rank, int size, const std::string& addr, int port, double timeout_s) : r_(rank), n_(size) {
  if (size < 1 || rank < 0 || rank >= size) throw std::runtime_error("TcpComm: bad rank/size");
  if (size == 1) return;
  // every rank >= 1 listens for its left neighbour on an ephemeral port of
  // the interface its control connection uses (not every interface: a stray
  // connection from elsewhere would be taken for the neighbour); rank 0
  // learns each rank's address from its control connection and publishes
  // (address, port) pairs, so the neighbour chain also forms across hosts
  int nb_lfd = -1, nb_port = 0;
  std::vector<uint32_t> nb_tab(2 * n_, 0);   // [2r] = IPv4 (network order), [2r+1] = port
  if (r_ == 0) {
    const int lfd = listen_on(addr, port, n_, nullptr);
    ctrl_.assign(n_, -1);
    for (int k = 1; k < n_; k++) {
      uint32_t peer = 0;
      const int fd = accept_one(lfd, timeout_s, &peer);
      int hello[2];
      recv_all(fd, hello, sizeof hello);
      if (hello[0] <= 0 || hello[0] >= n_ || ctrl_[hello[0]] >= 0) {
        ::close(lfd);
        throw std::runtime_error("TcpComm: bad or duplicate rank " + std::to_string(hello[0]));
      }
      ctrl_[hello[0]] = fd;
      nb_tab[2 * hello[0]] = peer;
      nb_tab[2 * hello[0] + 1] = (uint32_t)hello[1];
    }
    ::close(lfd);
    for (int k = 1; k < n_; k++) send_all(ctrl_[k], nb_tab.data(), sizeof(uint32_t) * nb_tab.size());
  } else {
    ctrl_.assign(1, connect_retry(addr, port, timeout_s));
    sockaddr_in me{};
    socklen_t ml = sizeof me;
    if (::getsockname(ctrl_[0], (sockaddr*)&me, &ml) != 0) fail("getsockname");
    char mine[INET_ADDRSTRLEN] = "0.0.0.0";
    ::inet_ntop(AF_INET, &me.sin_addr, mine, sizeof mine);
    nb_lfd = listen_on(mine, 0, 1, &nb_port);
    const int hello[2] = {r_, nb_port};
    send_all(ctrl_[0], hello, sizeof hello);
    recv_all(ctrl_[0], nb_tab.data(), sizeof(uint32_t) * nb_tab.size());
  }
  // neighbour chain: rank r connects to r+1's listener, r+1 accepts it
  if (r_ + 1 < n_) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)nb_tab[2 * (r_ + 1) + 1]);
    a.sin_addr.s_addr = nb_tab[2 * (r_ + 1)];
    char txt[INET_ADDRSTRLEN] = "?";
    ::inet_ntop(AF_INET, &a.sin_addr, txt, sizeof txt);
    right_ = connect_retry(a, txt, timeout_s);
    send_all(right_, &r_, sizeof r_);
  }
  if (r_ > 0) {
    left_ = accept_one(nb_lfd, timeout_s);
    int who = -1;
    recv_all(left_, &who, sizeof who);
    ::close(nb_lfd);
    if (who != r_ - 1) throw std::runtime_error("TcpComm: unexpected left neighbour " + std::to_string(who));
  }
  barrier();
}

TcpComm::~TcpComm() {
  for (int fd : ctrl_)
    if (fd >= 0) ::close(fd);
  if (left_ >= 0) ::close(left_);
  if (right_ >= 0) ::close(right_);
}

std::vector<std::string> TcpComm::allgather_bytes(const std::string& mine) {
  if (n_ == 1) return {mine};
  std::vector<std::string> all(n_);
  if (r_ == 0) {
    all[0] = mine;
    for (int k = 1; k < n_; k++) all[k] = recv_blob(ctrl_[k]);
    std::string pack;
    for (const auto& s : all) {
      const unsigned long long n = s.size();
      pack.append((const char*)&n, sizeof n);
      pack += s;
    }
    for (int k = 1; k < n_; k++) send_blob(ctrl_[k], pack);
  } else {
    send_blob(ctrl_[0], mine);
    const std::string pack = recv_blob(ctrl_[0]);
    size_t o = 0;
    for (int k = 0; k < n_; k++) {
      unsigned long long n = 0;
      if (o + sizeof n > pack.size()) throw std::runtime_error("TcpComm: short all-gather");
      std::memcpy(&n, pack.data() + o, sizeof n);
      o += sizeof n;
      all[k] = pack.substr(o, n);
      o += n;
    }
  }
  return all;
}

void TcpComm::send_to(int rank, const std::string& s) {
  if (r_ != 0 || rank <= 0 || rank >= n_) throw std::runtime_error("TcpComm::send_to: rank 0 to a rank >= 1 only");
  send_blob(ctrl_[rank], s);
}

std::string TcpComm::recv_from_root() {
  if (r_ == 0) throw std::runtime_error("TcpComm::recv_from_root on rank 0");
  return recv_blob(ctrl_[0]);
}

std::string TcpComm::broadcast(const std::string& s, int root) {
  const auto all = allgather_bytes(r_ == root ? s : std::string());
  return all[root];
}

namespace {
template <class T, class F>
T fold(TcpComm& c, T v, F f) {
  const auto all = c.allgather_bytes(std::string((const char*)&v, sizeof v));
  T acc;
  std::memcpy(&acc, all[0].data(), sizeof acc);
  for (size_t k = 1; k < all.size(); k++) {
    T x;
    std::memcpy(&x, all[k].data(), sizeof x);
    acc = f(acc, x);
  }
  return acc;
}
}  // namespace

real TcpComm::allreduce_min(real v) {
  return n_ == 1 ? v : fold<real>(*this, v, [](real a, real b) { return std::min(a, b); });
}
real TcpComm::allreduce_sum(real v) {
  return n_ == 1 ? v : fold<real>(*this, v, [](real a, real b) { return a + b; });
}
int TcpComm::allreduce_max_int(int v) {
  return n_ == 1 ? v : fold<int>(*this, v, [](int a, int b) { return std::max(a, b); });
}
void TcpComm::allreduce_residual(ResidualPack& p) {
  if (n_ == 1) return;
  p = fold<ResidualPack>(*this, p, [](ResidualPack a, const ResidualPack& b) {
    residual_merge_lex(a, b);
    return a;
  });
}

void TcpComm::neighbor_exchange(const void* to_left, void* from_left, size_t nleft, const void* to_right,
                                void* from_right, size_t nright) {
  struct Xfer {
    int fd;
    char* p;
    size_t left;
    bool send;
  };
  Xfer x[4];
  int nx = 0;
  if (nleft && left_ >= 0) {
    x[nx++] = {left_, (char*)to_left, nleft, true};
    x[nx++] = {left_, (char*)from_left, nleft, false};
  }
  if (nright && right_ >= 0) {
    x[nx++] = {right_, (char*)to_right, nright, true};
    x[nx++] = {right_, (char*)from_right, nright, false};
  }
  for (;;) {
    pollfd p[4];
    int np = 0, map[4];
    for (int k = 0; k < nx; k++)
      if (x[k].left) {
        p[np] = {x[k].fd, (short)(x[k].send ? POLLOUT : POLLIN), 0};
        map[np++] = k;
      }
    if (!np) return;
    const int rc = poll_retry(p, np, 300.0);
    if (rc == 0) throw std::runtime_error("TcpComm: halo exchange timed out");
    if (rc < 0) fail("halo exchange poll");
    for (int q = 0; q < np; q++) {
      if (!p[q].revents) continue;
      Xfer& t = x[map[q]];
      const ssize_t k = t.send ? ::send(t.fd, t.p, t.left, MSG_NOSIGNAL | MSG_DONTWAIT)
                               : ::recv(t.fd, t.p, t.left, MSG_DONTWAIT);
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) continue;
      if (k <= 0) fail("halo exchange");
      t.p += k;
      t.left -= (size_t)k;
    }
  }
}

RankEnv RankEnv::from_environ() {
  RankEnv e;
  auto geti = [](const char* k, int d) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : d;
  };
  e.rank = geti("RANK", 0);
  e.world = geti("WORLD_SIZE", 1);
  e.local_rank = geti("LOCAL_RANK", e.rank);
  e.port = geti("MASTER_PORT", 29613);
  if (const char* a = std::getenv("MASTER_ADDR")) e.addr = (*a && std::string(a) != "localhost") ? a : "127.0.0.1";
  return e;
}


}  // namespace hf2d
