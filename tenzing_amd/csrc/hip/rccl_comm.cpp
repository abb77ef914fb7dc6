#include "rccl_comm.hpp"

#include "core/util.hpp"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

namespace tz {

#define TZ_NCCL(x)                                                                                 \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) TZ_THROW(#x << " failed: " << ncclGetErrorString(r_));                  \
  } while (0)

namespace {
// live communicators, for the watchdog's abort-all (a communicator deregisters on destruction)
std::mutex g_mu;
std::vector<RcclComm *> g_live;
void register_comm(RcclComm *c) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_live.push_back(c);
}
void deregister_comm(RcclComm *c) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_live.erase(std::remove(g_live.begin(), g_live.end(), c), g_live.end());
}
} // namespace

int rccl_abort_all() {
  std::lock_guard<std::mutex> lk(g_mu);
  int n = 0;
  for (RcclComm *c : g_live)
    if (!c->aborted()) {
      c->abort();
      ++n;
    }
  return n;
}

bool rccl_multi_rank() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (RcclComm *c : g_live)
    if (c->size() > 1 && !c->aborted()) return true;
  return false;
}

namespace {
// ncclCommInitRank blocks until every rank has joined. A rank that failed before joining (or a
// bootstrap that cannot connect) would leave the others blocked forever, and a blocked init has
// no handle to abort. So the init runs on a helper thread (with this thread's device) and the
// caller waits with a bound (env TZ_RCCL_INIT_S, default 120 s): on timeout the caller raises,
// the collective agreement that follows drops RCCL, and the helper is abandoned. An abandoned
// helper whose init still completes (a late rank joined after all) aborts the communicator it
// got, so nothing unregistered keeps RCCL proxy threads and device resources alive.
struct InitState {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  bool abandoned = false; // the caller gave up waiting: the helper owns the outcome
  ncclResult_t res = ncclSuccess;
  ncclComm_t comm = nullptr;
};

ncclComm_t init_bounded(int nranks, const ncclUniqueId &id, int rank) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) TZ_THROW("hipGetDevice failed");
  double limit = 120.0;
  if (const char *v = std::getenv("TZ_RCCL_INIT_S")) limit = std::atof(v);
  auto st = std::make_shared<InitState>();
  std::thread([st, dev, nranks, id, rank] {
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclSuccess;
    if (hipSetDevice(dev) != hipSuccess) r = ncclSystemError;
    else r = ncclCommInitRank(&c, nranks, id, rank);
    std::unique_lock<std::mutex> lk(st->mu);
    if (st->abandoned) {
      lk.unlock();
      if (r == ncclSuccess && c) ncclCommAbort(c); // nobody will ever use or free it
      return;
    }
    st->res = r;
    st->comm = c;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  if (!st->cv.wait_for(lk, std::chrono::microseconds(int64_t(limit * 1e6)), [&] { return st->done; })) {
    st->abandoned = true;
    TZ_THROW("ncclCommInitRank did not complete within " << limit << " s (a rank missing?)");
  }
  if (st->res != ncclSuccess)
    TZ_THROW("ncclCommInitRank failed: " << ncclGetErrorString(st->res));
  return st->comm;
}
} // namespace

static ncclDataType_t dt(int dtype) {
  switch (dtype) {
  case 0: return ncclFloat32;
  case 1: return ncclFloat64;
  case 2: return ncclInt32;
  case 3: return ncclFloat16;
  case 4: return ncclBfloat16;
  case 5: return ncclInt64;
  case 6: return ncclUint8;
  default: TZ_THROW("bad dtype " << dtype);
  }
}

static ncclRedOp_t red_op(int red) {
  switch (red) {
  case RcclComm::Sum: return ncclSum;
  case RcclComm::Prod: return ncclProd;
  case RcclComm::Max: return ncclMax;
  case RcclComm::Min: return ncclMin;
  default: TZ_THROW("bad reduction " << red);
  }
}

size_t RcclComm::dtype_size(int dtype) {
  static const size_t sz[] = {4, 8, 4, 2, 2, 8, 1};
  TZ_CHECK(dtype >= 0 && dtype < 7, "bad dtype " << dtype);
  return sz[dtype];
}

RcclComm::RcclComm(Ctrl &ctrl, int device) : rank_(ctrl.rank()), size_(ctrl.size()) {
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess) TZ_THROW("hipSetDevice failed");
  }
  ncclUniqueId id;
  std::string s(sizeof(id), '\0');
  if (rank_ == 0) {
    TZ_NCCL(ncclGetUniqueId(&id));
    std::memcpy(&s[0], &id, sizeof(id));
  }
  ctrl.bcast(s, 0);
  std::memcpy(&id, s.data(), sizeof(id));
  comm_ = init_bounded(size_, id, rank_);
  register_comm(this);
}

RcclComm::RcclComm(const std::string &uniqueId, int rank, int size, int device)
    : rank_(rank), size_(size) {
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess) TZ_THROW("hipSetDevice failed");
  }
  ncclUniqueId id;
  TZ_CHECK(uniqueId.size() == sizeof(id), "bad RCCL unique id");
  std::memcpy(&id, uniqueId.data(), sizeof(id));
  comm_ = init_bounded(size_, id, rank_);
  register_comm(this);
}

RcclComm::~RcclComm() {
  deregister_comm(this);
  // an aborted communicator has already released its resources
  if (comm_ && !aborted_.load()) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::abort() {
  bool expected = false;
  if (!aborted_.compare_exchange_strong(expected, true)) return;
  if (comm_) ncclCommAbort(static_cast<ncclComm_t>(comm_));
}

void RcclComm::check_live() const {
  TZ_CHECK(!aborted_.load(), "RCCL communicator was aborted (watchdog)");
}

void RcclComm::sendrecv(const void *sendBuf, size_t sendCount, int sendPeer, void *recvBuf,
                        size_t recvCount, int recvPeer, int dtype, void *stream) const {
  check_live();
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  hipStream_t s = static_cast<hipStream_t>(stream);
  TZ_NCCL(ncclGroupStart());
  if (sendCount) TZ_NCCL(ncclSend(sendBuf, sendCount, dt(dtype), sendPeer, c, s));
  if (recvCount) TZ_NCCL(ncclRecv(recvBuf, recvCount, dt(dtype), recvPeer, c, s));
  TZ_NCCL(ncclGroupEnd());
}

void RcclComm::exchange(const std::vector<Xfer> &xs, int dtype, void *stream) const {
  check_live();
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  hipStream_t s = static_cast<hipStream_t>(stream);
  TZ_NCCL(ncclGroupStart());
  for (const auto &x : xs) {
    if (x.sendCount) TZ_NCCL(ncclSend(x.send, x.sendCount, dt(dtype), x.sendPeer, c, s));
    if (x.recvCount) TZ_NCCL(ncclRecv(x.recv, x.recvCount, dt(dtype), x.recvPeer, c, s));
  }
  TZ_NCCL(ncclGroupEnd());
}

void RcclComm::allreduce_sum(void *buf, size_t count, int dtype, void *stream) const {
  check_live();
  TZ_NCCL(ncclAllReduce(buf, buf, count, dt(dtype), ncclSum, static_cast<ncclComm_t>(comm_),
                        static_cast<hipStream_t>(stream)));
}

void RcclComm::allreduce(const void *send, void *recv, size_t count, int dtype, int red,
                         void *stream) const {
  check_live();
  TZ_NCCL(ncclAllReduce(send, recv, count, dt(dtype), red_op(red), static_cast<ncclComm_t>(comm_),
                        static_cast<hipStream_t>(stream)));
}

void RcclComm::allgather(const void *send, void *recv, size_t count, int dtype, void *stream) const {
  check_live();
  TZ_NCCL(ncclAllGather(send, recv, count, dt(dtype), static_cast<ncclComm_t>(comm_),
                        static_cast<hipStream_t>(stream)));
}

void RcclComm::reduce_scatter(const void *send, void *recv, size_t recvCount, int dtype, int red,
                              void *stream) const {
  check_live();
  TZ_NCCL(ncclReduceScatter(send, recv, recvCount, dt(dtype), red_op(red),
                            static_cast<ncclComm_t>(comm_), static_cast<hipStream_t>(stream)));
}

void RcclComm::broadcast(const void *send, void *recv, size_t count, int root, int dtype,
                         void *stream) const {
  check_live();
  TZ_CHECK(root >= 0 && root < size_, "broadcast root " << root << " out of range");
  TZ_NCCL(ncclBroadcast(send, recv, count, dt(dtype), root, static_cast<ncclComm_t>(comm_),
                        static_cast<hipStream_t>(stream)));
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  TZ_NCCL(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char *>(&id), sizeof(id));
}

std::string RcclComm::version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v);
}

std::vector<std::shared_ptr<RcclComm>> make_rccl_comms(Ctrl &ctrl, int device, int n) {
  // one broadcast carries every unique id (a control-plane round trip per communicator adds
  // up at 26 directions), then every rank initializes the communicators in the same order
  ncclUniqueId id;
  std::string ids(sizeof(id) * size_t(std::max(n, 0)), '\0');
  if (ctrl.rank() == 0) {
    for (int i = 0; i < n; ++i) {
      TZ_NCCL(ncclGetUniqueId(&id));
      std::memcpy(&ids[sizeof(id) * size_t(i)], &id, sizeof(id));
    }
  }
  ctrl.bcast(ids, 0);
  TZ_CHECK(ids.size() == sizeof(id) * size_t(std::max(n, 0)), "unique-id broadcast truncated");
  std::vector<std::shared_ptr<RcclComm>> out;
  for (int i = 0; i < n; ++i)
    out.push_back(std::make_shared<RcclComm>(ids.substr(sizeof(id) * size_t(i), sizeof(id)),
                                             ctrl.rank(), ctrl.size(), device));
  return out;
}

} // namespace tz
