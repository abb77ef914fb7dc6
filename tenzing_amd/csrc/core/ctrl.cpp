#include "ctrl.hpp"
#include "util.hpp"

#include <arpa/inet.h>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/select.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <thread>
#include <unistd.h>

namespace tz {

std::vector<std::string> Ctrl::alltoallv(const std::vector<std::string> &out) {
  TZ_CHECK(int(out.size()) == size(), "alltoallv: " << out.size() << " payloads for " << size() << " ranks");
  // pack [u64 length][bytes] per destination, allgather, keep the parts addressed to me
  std::string packed;
  for (const auto &o : out) {
    const uint64_t n = o.size();
    packed.append(reinterpret_cast<const char *>(&n), sizeof(n));
    packed += o;
  }
  const std::vector<std::string> all = allgather(packed);
  std::vector<std::string> in(all.size());
  for (size_t src = 0; src < all.size(); ++src) {
    size_t at = 0;
    for (int dst = 0; dst < size(); ++dst) {
      uint64_t n = 0;
      TZ_CHECK(at + sizeof(n) <= all[src].size(), "alltoallv: truncated payload from rank " << src);
      std::memcpy(&n, all[src].data() + at, sizeof(n));
      at += sizeof(n);
      TZ_CHECK(at + n <= all[src].size(), "alltoallv: truncated payload from rank " << src);
      if (dst == rank()) in[src] = all[src].substr(at, n);
      at += n;
    }
  }
  return in;
}

int64_t Ctrl::bcast_int(int64_t v, int root) {
  std::string s(reinterpret_cast<const char *>(&v), sizeof(v));
  bcast(s, root);
  std::memcpy(&v, s.data(), sizeof(v));
  return v;
}

namespace {
void send_all(int fd, const void *buf, size_t n) {
  const char *p = static_cast<const char *>(buf);
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      TZ_THROW("ctrl send failed: " << std::strerror(errno));
    }
    p += w;
    n -= size_t(w);
  }
}
void recv_all(int fd, void *buf, size_t n) {
  char *p = static_cast<char *>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK)
        // the peer's socket timeout (TZ_CTRL_TIMEOUT_S): a rank stuck outside every watchdog
        // ends the job with this message instead of leaving every other rank blocked silently
        TZ_THROW("ctrl: no message from a peer rank within the control-plane timeout "
                 "(TZ_CTRL_TIMEOUT_S); that rank is hung or gone");
      TZ_THROW("ctrl recv failed: " << std::strerror(errno));
    }
    if (r == 0) TZ_THROW("ctrl peer closed connection");
    p += r;
    n -= size_t(r);
  }
}
void send_frame(int fd, const std::string &s) {
  uint64_t n = s.size();
  send_all(fd, &n, sizeof(n));
  if (n) send_all(fd, s.data(), n);
}
std::string recv_frame(int fd) {
  uint64_t n = 0;
  recv_all(fd, &n, sizeof(n));
  std::string s(n, '\0');
  if (n) recv_all(fd, &s[0], n);
  return s;
}
void nodelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
/// the other end of `fd` has closed it (readable at end of file, or reset): a peer that left
bool peer_closed(int fd) {
  pollfd p{fd, POLLIN, 0};
  if (::poll(&p, 1, 0) <= 0) return false; // nothing pending: still open
  if (p.revents & (POLLHUP | POLLERR | POLLNVAL)) return true;
  char c;
  const ssize_t r = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
  return r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK);
}
/// default receive timeout of a joined peer socket: env TZ_CTRL_TIMEOUT_S (default 900 s: above
/// any search step, below "forever"; 0 = none). Runs whose watchdog budget is longer raise it
/// (TcpCtrl::ensure_timeout, called by the benchmarker before every run)
double default_peer_timeout() {
  double t = 900.0;
  if (const char *v = std::getenv("TZ_CTRL_TIMEOUT_S")) t = std::atof(v);
  return t > 0 ? t : 0.0;
}
void set_rcv_timeout(int fd, double t) {
  timeval tv{};
  tv.tv_sec = long(t);
  tv.tv_usec = long((t - double(tv.tv_sec)) * 1e6);
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}
} // namespace

TcpCtrl::TcpCtrl(int rank, int size) : rank_(rank), size_(size), peers_(size, -1) {
  TZ_CHECK(size >= 1 && rank >= 0 && rank < size, "bad rank/size " << rank << "/" << size);
}

TcpCtrl::~TcpCtrl() {
  for (int fd : peers_)
    if (fd >= 0) ::close(fd);
  if (listenFd_ >= 0) ::close(listenFd_);
}

int TcpCtrl::listen(int port, const std::string &bindAddr) {
  TZ_CHECK(rank_ == 0, "only rank 0 listens");
  listenFd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  TZ_CHECK(listenFd_ >= 0, "socket: " << std::strerror(errno));
  int one = 1;
  ::setsockopt(listenFd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(uint16_t(port));
  TZ_CHECK(::inet_pton(AF_INET, bindAddr.c_str(), &addr.sin_addr) == 1, "bad bind addr");
  TZ_CHECK(::bind(listenFd_, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) == 0,
           "bind: " << std::strerror(errno));
  TZ_CHECK(::listen(listenFd_, 256) == 0, "listen: " << std::strerror(errno));
  socklen_t len = sizeof(addr);
  ::getsockname(listenFd_, reinterpret_cast<sockaddr *>(&addr), &len);
  return ntohs(addr.sin_port);
}

namespace {
constexpr uint32_t kHello = 0x545a4331;   // "TZC1": a peer rank's first frame
constexpr uint32_t kAck = 0x545a4143;     // "TZAC": rank 0 took the peer (sent at once)
constexpr uint32_t kWelcome = 0x545a4f4b; // "TZOK": rank 0's release (once every rank joined)
struct Hello {
  uint32_t magic;
  int32_t size, rank;
  int32_t job; // the job's base port (rendezvous): a rank 0 of another job does not take it
};
} // namespace

int TcpCtrl::connect_acked(const std::string &host, int port, std::string &why) const {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  TZ_CHECK(::getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) == 0, "getaddrinfo " << host);
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  const int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0) {
    ::close(fd);
    return -1;
  }
  nodelay(fd);
  // rank 0 acknowledges a peer at once; a listener that does not (another program that holds
  // the port) is left, not waited on forever. Rank 0 may first have to drop a backlog of stray
  // connections (up to 1 s each), so the wait is generous; a peer that gives up anyway comes
  // back and rank 0 replaces its closed connection
  timeval ack{15, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &ack, sizeof(ack));
  uint32_t a = 0;
  try {
    const Hello h{kHello, size_, rank_, job_};
    send_all(fd, &h, sizeof(h));
    recv_all(fd, &a, sizeof(a));
  } catch (const Error &) {
    a = 0;
  }
  if (a == kAck) return fd;
  why = "a listener on port " + ps + " that is not this job's rank 0";
  ::close(fd);
  return -1;
}

void TcpCtrl::connect(const std::string &host, int port, double timeoutS) {
  if (size_ == 1) return;
  if (rank_ == 0) {
    TZ_CHECK(listenFd_ >= 0, "rank 0 must listen() before connect()");
    const double t0 = wtime();
    for (int joined = 1;;) {
      if (joined == size_) {
        // every rank joined; a peer that has since closed its connection (it gave up waiting
        // for the acknowledgement and will come back) is waited for again
        for (int i = 1; i < size_; ++i)
          if (peers_[i] >= 0 && peer_closed(peers_[i])) {
            ::close(peers_[i]);
            peers_[i] = -1;
            --joined;
            TZ_LOG(Info, "ctrl rendezvous: rank " << i << " left before the release; waiting for it again");
          }
        if (joined == size_) break;
      }
      // bounded: a rank that never comes must not leave rank 0 blocked in accept() forever
      timeval tv{};
      const double left = timeoutS - (wtime() - t0);
      TZ_CHECK(left > 0, "ctrl rendezvous: " << (size_ - joined) << " of " << size_ - 1
                                              << " ranks did not connect within " << timeoutS << " s");
      tv.tv_sec = long(left);
      tv.tv_usec = long((left - double(tv.tv_sec)) * 1e6);
      fd_set rd;
      FD_ZERO(&rd);
      FD_SET(listenFd_, &rd);
      const int sel = ::select(listenFd_ + 1, &rd, nullptr, nullptr, &tv);
      if (sel < 0 && errno == EINTR) continue;
      TZ_CHECK(sel >= 0, "select: " << std::strerror(errno));
      if (sel == 0) continue; // timed out: the check above reports it
      int fd = ::accept(listenFd_, nullptr, nullptr);
      TZ_CHECK(fd >= 0, "accept: " << std::strerror(errno));
      nodelay(fd);
      // a connection that does not speak the handshake within a second is dropped
      timeval hs{1, 0};
      ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &hs, sizeof(hs));
      Hello h{};
      try {
        recv_all(fd, &h, sizeof(h));
      } catch (const Error &) {
        h.magic = 0;
      }
      timeval none{0, 0};
      ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
      if (h.magic != kHello || h.job != job_) {
        // not this job: no acknowledgement, so the peer moves on to the next candidate port
        ::close(fd);
        TZ_LOG(Warn, "ctrl rendezvous: dropped a connection "
                         << (h.magic != kHello ? "without the handshake" : "of another job"));
        continue;
      }
      if (h.size != size_ || h.rank <= 0 || h.rank >= size_) {
        ::close(fd);
        TZ_THROW("ctrl rendezvous: peer says rank " << h.rank << " of " << h.size << " (this job: "
                                                    << size_ << " ranks; a rank of another job?)");
      }
      if (peers_[h.rank] >= 0) {
        // the same rank again: a peer that gave up waiting for its acknowledgement (this loop
        // was held up by stray connections) closed the old connection and came back -- take
        // the new one; while the old one is still open, the new one is a stray and is dropped
        if (!peer_closed(peers_[h.rank])) {
          ::close(fd);
          TZ_LOG(Warn, "ctrl rendezvous: dropped a second connection of rank " << h.rank
                                                                                 << " (its first is open)");
          continue;
        }
        ::close(peers_[h.rank]);
        peers_[h.rank] = -1;
        --joined;
        TZ_LOG(Info, "ctrl rendezvous: rank " << h.rank << " reconnected");
      }
      peers_[h.rank] = fd;
      send_all(fd, &kAck, sizeof(kAck));
      ++joined;
    }
    // release everyone
    timeoutS_ = default_peer_timeout();
    for (int i = 1; i < size_; ++i) {
      send_all(peers_[i], &kWelcome, sizeof(kWelcome));
      if (timeoutS_ > 0) set_rcv_timeout(peers_[i], timeoutS_);
    }
    return;
  }
  const double t0 = wtime();
  int fd = -1;
  std::string lastWhy = "connection refused";
  // every candidate port in turn (rendezvous: rank 0 took the first one it could bind), until
  // one answers as this job's rank 0
  const int nports = std::max(1, connectPorts_);
  for (int k = 0;; k = (k + 1) % nports) {
    fd = connect_acked(host, port + k, lastWhy);
    if (fd >= 0) break;
    if (wtime() - t0 > timeoutS)
      TZ_THROW("ctrl connect to " << host << ":" << port
                                  << (nports > 1 ? "+" + std::to_string(nports - 1) : std::string())
                                  << " timed out (" << lastWhy << ")");
    if (k == nports - 1) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  // the release comes once every rank joined: wait for it as long as the rendezvous may take
  const double left = std::max(1.0, timeoutS - (wtime() - t0));
  timeval rel{};
  rel.tv_sec = long(left);
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &rel, sizeof(rel));
  uint32_t w = 0;
  recv_all(fd, &w, sizeof(w));
  TZ_CHECK(w == kWelcome, "ctrl rendezvous: " << host << ":" << port << " is not this job's rank 0");
  timeval none{0, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
  timeoutS_ = default_peer_timeout();
  if (timeoutS_ > 0) set_rcv_timeout(fd, timeoutS_);
  peers_[0] = fd;
}

void TcpCtrl::ensure_timeout(double seconds) {
  if (timeoutS_ <= 0 || seconds <= timeoutS_) return; // no timeout at all, or long enough
  timeoutS_ = seconds;
  for (int fd : peers_)
    if (fd >= 0) set_rcv_timeout(fd, timeoutS_);
}

void TcpCtrl::rendezvous(const std::string &host, int port, double timeoutS, int nports) {
  TZ_CHECK(port > 0 && port + nports - 1 < 65536 && nports >= 1,
           "ctrl rendezvous ports " << port << "+" << nports - 1 << " out of range");
  if (size_ == 1) return;
  if (rank_ == 0) {
    // the first of the candidate ports that is free (another program may hold one); the other
    // ranks try them all, and only this job's rank 0 acknowledges them
    std::string errs;
    for (int k = 0; k < nports && listenFd_ < 0; ++k) {
      try {
        listen(port + k, "0.0.0.0");
      } catch (const Error &e) {
        if (listenFd_ >= 0) ::close(listenFd_);
        listenFd_ = -1;
        errs += std::string("\n  ") + e.what();
      }
    }
    TZ_CHECK(listenFd_ >= 0, "ctrl rendezvous: none of ports " << port << ".." << port + nports - 1
                                                               << " could be bound:" << errs);
  }
  connectPorts_ = nports;
  job_ = port;
  connect(host, port, timeoutS);
  connectPorts_ = 1;
}

void TcpCtrl::rendezvous_file(const std::string &path, const std::string &host, double timeoutS) {
  if (rank_ == 0) {
    int port = listen(0);
    const std::string tmp = path + ".tmp";
    {
      std::ofstream f(tmp);
      f << port << "\n";
    }
    ::rename(tmp.c_str(), path.c_str());
    connect(host, port, timeoutS);
  } else {
    const double t0 = wtime();
    int port = 0;
    while (true) {
      std::ifstream f(path);
      if (f && (f >> port) && port > 0) break;
      TZ_CHECK(wtime() - t0 < timeoutS, "rendezvous file " << path << " never appeared");
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    connect(host, port, timeoutS);
  }
}

void TcpCtrl::barrier() {
  if (size_ == 1) return;
  char c = 0;
  if (rank_ == 0) {
    for (int i = 1; i < size_; ++i) recv_all(peers_[i], &c, 1);
    for (int i = 1; i < size_; ++i) send_all(peers_[i], &c, 1);
  } else {
    send_all(peers_[0], &c, 1);
    recv_all(peers_[0], &c, 1);
  }
}

void TcpCtrl::bcast(std::string &data, int root) {
  if (size_ == 1) return;
  if (root != 0) {
    if (rank_ == root) send_frame(peers_[0], data);
    else if (rank_ == 0) data = recv_frame(peers_[root]);
  }
  if (rank_ == 0) {
    for (int i = 1; i < size_; ++i)
      if (i != root) send_frame(peers_[i], data);
  } else if (rank_ != root) {
    data = recv_frame(peers_[0]);
  }
}

void TcpCtrl::allreduce(double *v, size_t n, bool isMax) {
  if (size_ == 1) return;
  std::string buf(reinterpret_cast<const char *>(v), n * sizeof(double));
  if (rank_ == 0) {
    std::vector<double> tmp(n);
    for (int i = 1; i < size_; ++i) {
      std::string f = recv_frame(peers_[i]);
      TZ_CHECK(f.size() == n * sizeof(double), "allreduce size mismatch");
      std::memcpy(tmp.data(), f.data(), f.size());
      for (size_t k = 0; k < n; ++k) v[k] = isMax ? std::max(v[k], tmp[k]) : v[k] + tmp[k];
    }
    std::string out(reinterpret_cast<const char *>(v), n * sizeof(double));
    for (int i = 1; i < size_; ++i) send_frame(peers_[i], out);
  } else {
    send_frame(peers_[0], buf);
    std::string f = recv_frame(peers_[0]);
    TZ_CHECK(f.size() == n * sizeof(double), "allreduce size mismatch (mismatched collectives?)");
    std::memcpy(v, f.data(), n * sizeof(double));
  }
}

void TcpCtrl::allreduce_max(double *v, size_t n) { allreduce(v, n, true); }
void TcpCtrl::allreduce_sum(double *v, size_t n) { allreduce(v, n, false); }

std::vector<std::string> TcpCtrl::allgather(const std::string &mine) {
  std::vector<std::string> all(size_);
  all[rank_] = mine;
  if (size_ == 1) return all;
  if (rank_ == 0) {
    for (int i = 1; i < size_; ++i) all[i] = recv_frame(peers_[i]);
    for (int i = 1; i < size_; ++i)
      for (int k = 0; k < size_; ++k) send_frame(peers_[i], all[k]);
  } else {
    send_frame(peers_[0], mine);
    for (int k = 0; k < size_; ++k) all[k] = recv_frame(peers_[0]);
  }
  return all;
}

std::vector<std::string> TcpCtrl::alltoallv(const std::vector<std::string> &out) {
  TZ_CHECK(int(out.size()) == size_, "alltoallv: " << out.size() << " payloads for " << size_ << " ranks");
  std::vector<std::string> in(size_);
  if (size_ == 1) {
    in[0] = out[0];
    return in;
  }
  if (rank_ == 0) {
    // the hub: every rank's payloads in, then each destination gets its column, by source
    std::vector<std::vector<std::string>> m(size_, std::vector<std::string>(size_));
    m[0] = out;
    for (int i = 1; i < size_; ++i)
      for (int k = 0; k < size_; ++k) m[i][k] = recv_frame(peers_[i]);
    for (int j = 1; j < size_; ++j)
      for (int i = 0; i < size_; ++i) send_frame(peers_[j], m[i][j]);
    for (int i = 0; i < size_; ++i) in[i] = std::move(m[i][0]);
  } else {
    for (int k = 0; k < size_; ++k) send_frame(peers_[0], out[k]);
    for (int i = 0; i < size_; ++i) in[i] = recv_frame(peers_[0]);
  }
  return in;
}

} // namespace tz
