// Host control plane: the tiny, latency-bound collectives the search needs (stop flags,
// schedule broadcast, barrier, max-reduction of timings).
//
// Parity: the reference uses MPI for these (MPI_Bcast of the schedule JSON, src/sequence.cpp:
// 88-125; MPI_Barrier/MPI_Allreduce(MAX) in src/benchmarker.cpp:45-145; Stop-flag MPI_Bcast in
// tenzing-mcts mcts.hpp:149-150 and tenzing-dfs dfs.hpp:67-68). The GPU data plane is RCCL, so
// the default control plane is a native TCP star (rank 0 hub, TCP_NODELAY, length-prefixed
// frames) bootstrapped from the launcher's rendezvous (torchrun). Programs started by an MPI
// launcher, as the reference's are, can use MpiCtrl instead (host MPI, opened at run time). Neither
// is on the device path: candidate schedules move their payloads over RCCL/xGMI.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace tz {

class Ctrl {
public:
  virtual ~Ctrl() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual void barrier() = 0;
  virtual void bcast(std::string &data, int root) = 0;
  virtual void allreduce_max(double *v, size_t n) = 0;
  virtual void allreduce_sum(double *v, size_t n) = 0;
  /// every rank gets every rank's string
  virtual std::vector<std::string> allgather(const std::string &mine) = 0;
  /// personalized exchange: out[j] goes to rank j; returns in[i] = what rank i sent to me. The
  /// generic version allgathers everything (correct for any control plane, but every rank
  /// receives every payload); TcpCtrl routes each payload to its destination only.
  virtual std::vector<std::string> alltoallv(const std::vector<std::string> &out);

  double allreduce_max(double v) {
    allreduce_max(&v, 1);
    return v;
  }
  int64_t bcast_int(int64_t v, int root);
  /// a collective may wait at least `seconds` for the other ranks before it declares one of them
  /// gone (control planes with a receive timeout raise it; never lowered)
  virtual void ensure_timeout(double seconds) { (void)seconds; }
};

class SelfCtrl : public Ctrl {
public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  void barrier() override {}
  void bcast(std::string &, int) override {}
  void allreduce_max(double *, size_t) override {}
  void allreduce_sum(double *, size_t) override {}
  std::vector<std::string> allgather(const std::string &mine) override { return {mine}; }
  std::vector<std::string> alltoallv(const std::vector<std::string> &out) override { return out; }
};

class TcpCtrl : public Ctrl {
public:
  TcpCtrl(int rank, int size);
  ~TcpCtrl() override;
  TcpCtrl(const TcpCtrl &) = delete;
  TcpCtrl &operator=(const TcpCtrl &) = delete;

  /// rank 0 only: bind and listen (port 0 = ephemeral); returns the bound port
  int listen(int port = 0, const std::string &bindAddr = "0.0.0.0");
  /// rank 0: accept size-1 peers; others: connect (retrying until timeout)
  void connect(const std::string &host, int port, double timeoutS = 300.0);
  /// rank 0 writes its port to `path`; others poll the file (CLI bootstrap without Python)
  void rendezvous_file(const std::string &path, const std::string &host, double timeoutS = 300.0);
  /// rank 0 listens on `port` of every interface, the others connect to host:port (retrying
  /// until rank 0 is up): a launcher-style rendezvous with no store and no torch.distributed.
  /// Every connection carries a handshake (magic, world size, rank), so a stray connection to
  /// the port is dropped instead of taken for a rank.
  /// `nports` candidate ports from `port` on: rank 0 listens on the first it can bind
  void rendezvous(const std::string &host, int port, double timeoutS = 300.0, int nports = 8);

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void barrier() override;
  void bcast(std::string &data, int root) override;
  void allreduce_max(double *v, size_t n) override;
  void allreduce_sum(double *v, size_t n) override;
  std::vector<std::string> allgather(const std::string &mine) override;
  std::vector<std::string> alltoallv(const std::vector<std::string> &out) override;
  using Ctrl::allreduce_max;
  /// raise every peer socket's receive timeout to `seconds` if it is lower (0 = none: stays)
  void ensure_timeout(double seconds) override;
  /// the peer sockets' receive timeout in seconds (0 = none)
  double timeout() const { return timeoutS_; }

private:
  void allreduce(double *v, size_t n, bool isMax);
  double timeoutS_ = 0; // receive timeout of the joined peer sockets (0 = none)
  /// one connection attempt to host:port with the handshake; the fd, or -1 (`why` updated)
  int connect_acked(const std::string &host, int port, std::string &why) const;
  int connectPorts_ = 1; // candidate ports connect() cycles through (rendezvous)
  int32_t job_ = 0;      // job token of the handshake (rendezvous: the base port; else 0)
  int rank_, size_;
  int listenFd_ = -1;
  std::vector<int> peers_; // rank 0: fd per rank (index 0 unused); others: peers_[0] = root
};

/// Control plane over MPI_COMM_WORLD for ranks started by mpirun / mpiexec / srun (the
/// reference's launch model). libmpi (MPICH ABI) is opened at run time: $TZ_MPI_LIB, the
/// loader's libmpi.so.12 / libmpi.so, then /opt/conda/lib. MPI_Init_thread runs unless MPI is
/// already initialized, and MPI_Finalize then runs at process exit.
class MpiCtrl : public Ctrl {
public:
  explicit MpiCtrl(const std::string &lib = "");
  /// ranks an MPICH-family launcher started (PMI / PMIx / MVAPICH environment), 1 if none
  static int launcher_size();
  /// this process is one of several ranks started by an MPI launcher
  static bool launched();
  /// the node-local rank the launcher exported, -1 if none
  static int launcher_local_rank();
  /// path of the MPI library in use
  std::string library() const;

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void barrier() override;
  void bcast(std::string &data, int root) override;
  void allreduce_max(double *v, size_t n) override;
  void allreduce_sum(double *v, size_t n) override;
  std::vector<std::string> allgather(const std::string &mine) override;
  std::vector<std::string> alltoallv(const std::vector<std::string> &out) override;
  using Ctrl::allreduce_max;

private:
  int rank_ = 0, size_ = 1;
};

} // namespace tz
