// Native rank bootstrap and host communicator for one-process-per-rank runs of
// bin/hf2d (no Python, no MPI).
//
// The reference initialises MPI inside main and splits the grid among the
// ranks there (hf2d_start.cpp:79-289; launched by bin/OpenHyperFLOW2D.sh with
// mpiexec).  Here the environment torchrun / OpenHyperFLOW2D.sh sets --
// RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT -- drives a TCP
// rendezvous at rank 0:
//   * a control star (every rank <-> rank 0) carries the collectives of the
//     driver (all-gather of variable-size blobs; min/sum/max and the residual
//     reduction are folded from it in rank order, so every rank computes the
//     same bits), the RCCL unique id and the p2p mailbox descriptors;
//   * a chain of neighbour sockets (rank r <-> r+1) carries the halo columns
//     of the CPU backend (the GPU backend exchanges halos over xGMI p2p or
//     RCCL instead).
#pragma once

#include <string>
#include <vector>

#include "solver.hpp"

namespace hf2d {

class TcpComm : public Comm {
 public:
  // rank 0 listens on addr:port; the others connect (retrying until
  // timeout_s) and report their neighbour listener.
  TcpComm(int rank, int size, const std::string& addr, int port, double timeout_s = 300.0);
  ~TcpComm() override;
  TcpComm(const TcpComm&) = delete;
  TcpComm& operator=(const TcpComm&) = delete;

  int rank() const override { return r_; }
  int size() const override { return n_; }
  real allreduce_min(real v) override;
  real allreduce_sum(real v) override;
  int allreduce_max_int(int v) override;
  void allreduce_residual(ResidualPack& p) override;
  std::vector<std::string> allgather_bytes(const std::string& mine) override;
  std::string broadcast(const std::string& s, int root = 0);
  // point-to-point with rank 0 over the control connection (strip scatter)
  void send_to(int rank, const std::string& s);   // rank 0 only
  std::string recv_from_root();                    // ranks >= 1

  // Full-duplex exchange with the strip neighbours (either side may be
  // absent: pass nbytes 0).  Sends and receives proceed together, so
  // arbitrarily large columns cannot deadlock on socket buffers.
  void neighbor_exchange(const void* to_left, void* from_left, size_t nleft, const void* to_right, void* from_right,
                         size_t nright);

 private:
  int r_, n_;
  std::vector<int> ctrl_;   // rank 0: fd of each rank (index = rank); others: ctrl_[0] = fd to rank 0
  int left_ = -1, right_ = -1;
};

// RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT (torchrun names)
struct RankEnv {
  int rank = 0, world = 1, local_rank = 0;
  std::string addr = "127.0.0.1";
  int port = 29613;
  static RankEnv from_environ();
};


}  // namespace hf2d
