#include "comm_ops.hpp"

#include "core/util.hpp"

#include <algorithm>

namespace tz {

CommOp::CommOp(std::string name, CommSet comms, int dtype, std::shared_ptr<void> keep)
    : name_(std::move(name)), comms_(std::move(comms)), dtype_(dtype), keep_(std::move(keep)) {
  TZ_CHECK(!comms_.empty(), name_ << ": needs at least one communicator");
  for (const auto &c : comms_) {
    TZ_CHECK(c, name_ << ": null communicator");
    TZ_CHECK(c->size() == comms_[0]->size() && c->rank() == comms_[0]->rank(),
             name_ << ": communicators must span the same ranks");
  }
  (void)RcclComm::dtype_size(dtype_); // validates
}

Json CommOp::json() const {
  Json j;
  j["name"] = name_;
  j["kind"] = kind();
  return j;
}

int CommOp::nranks() const { return comms_[0]->size(); }

const RcclComm &CommOp::comm_for(void *stream, Executor &ex) const {
  const int k = std::max(ex.stream_index(stream), 0);
  return *comms_[size_t(k) % comms_.size()];
}

static void check_peer(const std::string &op, int peer, int n) {
  TZ_CHECK(peer >= 0 && peer < n, op << ": peer " << peer << " outside [0, " << n << ")");
}

// ------------------------------------------------------------------ point-to-point

SendRecvOp::SendRecvOp(std::string name, CommSet comms, const void *send, size_t send_count,
                       int send_peer, void *recv, size_t recv_count, int recv_peer, int dtype,
                       std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), send_(send),
      send_count_(send_count), send_peer_(send_peer), recv_(recv), recv_count_(recv_count),
      recv_peer_(recv_peer) {
  if (send_count_) {
    TZ_CHECK(send_, this->name() << ": null send buffer");
    check_peer(this->name(), send_peer_, nranks());
  }
  if (recv_count_) {
    TZ_CHECK(recv_, this->name() << ": null receive buffer");
    check_peer(this->name(), recv_peer_, nranks());
  }
}

void SendRecvOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).sendrecv(send_, send_count_, send_peer_, recv_, recv_count_, recv_peer_,
                                dtype(), stream);
}

AlltoallvOp::AlltoallvOp(std::string name, CommSet comms, std::vector<RcclComm::Xfer> xfers,
                         int dtype, std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), xfers_(std::move(xfers)) {
  for (const auto &x : xfers_) {
    if (x.sendCount) {
      TZ_CHECK(x.send, this->name() << ": null send buffer");
      check_peer(this->name(), x.sendPeer, nranks());
    }
    if (x.recvCount) {
      TZ_CHECK(x.recv, this->name() << ": null receive buffer");
      check_peer(this->name(), x.recvPeer, nranks());
    }
  }
}

double AlltoallvOp::bytes() const {
  double b = 0;
  for (const auto &x : xfers_) b += double(x.sendCount + x.recvCount) * double(esize());
  return b;
}

double AlltoallvOp::cost_us() const {
  // peers are reached over separate xGMI links: the largest single transfer bounds the op
  size_t m = 0;
  for (const auto &x : xfers_) m = std::max({m, x.sendCount, x.recvCount});
  return link_cost_us(double(m) * double(esize()));
}

void AlltoallvOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).exchange(xfers_, dtype(), stream);
}

// ------------------------------------------------------------------ collectives

AllReduceOp::AllReduceOp(std::string name, CommSet comms, const void *send, void *recv,
                         size_t count, int dtype, int red, std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), send_(send), recv_(recv),
      count_(count), red_(red) {
  TZ_CHECK(red_ >= RcclComm::Sum && red_ <= RcclComm::Min, this->name() << ": bad reduction");
  TZ_CHECK(!count_ || (send_ && recv_), this->name() << ": null buffer");
}

double AllReduceOp::cost_us() const {
  // ring: 2 (n-1)/n of the buffer crosses each link
  const double n = double(nranks());
  return link_cost_us(n > 1 ? 2.0 * (n - 1.0) / n * bytes() : 0.0, 10.0);
}

void AllReduceOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).allreduce(send_, recv_, count_, dtype(), red_, stream);
}

AllGatherOp::AllGatherOp(std::string name, CommSet comms, const void *send, void *recv,
                         size_t count, int dtype, std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), send_(send), recv_(recv),
      count_(count) {
  TZ_CHECK(!count_ || (send_ && recv_), this->name() << ": null buffer");
}

double AllGatherOp::cost_us() const {
  const double n = double(nranks());
  return link_cost_us((n - 1.0) / n * bytes(), 10.0);
}

void AllGatherOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).allgather(send_, recv_, count_, dtype(), stream);
}

ReduceScatterOp::ReduceScatterOp(std::string name, CommSet comms, const void *send, void *recv,
                                 size_t recv_count, int dtype, int red, std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), send_(send), recv_(recv),
      recv_count_(recv_count), red_(red) {
  TZ_CHECK(red_ >= RcclComm::Sum && red_ <= RcclComm::Min, this->name() << ": bad reduction");
  TZ_CHECK(!recv_count_ || (send_ && recv_), this->name() << ": null buffer");
}

double ReduceScatterOp::cost_us() const {
  const double n = double(nranks());
  return link_cost_us((n - 1.0) / n * bytes(), 10.0);
}

void ReduceScatterOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).reduce_scatter(send_, recv_, recv_count_, dtype(), red_, stream);
}

BroadcastOp::BroadcastOp(std::string name, CommSet comms, const void *send, void *recv,
                         size_t count, int root, int dtype, std::shared_ptr<void> keep)
    : CommOp(std::move(name), std::move(comms), dtype, std::move(keep)), send_(send), recv_(recv),
      count_(count), root_(root) {
  check_peer(this->name(), root_, nranks());
  TZ_CHECK(!count_ || recv_, this->name() << ": null receive buffer");
  TZ_CHECK(!count_ || this->comms()[0]->rank() != root_ || send_, this->name() << ": root needs a send buffer");
}

void BroadcastOp::launch(void *stream, Executor &ex) const {
  comm_for(stream, ex).broadcast(send_, recv_, count_, root_, dtype(), stream);
}

} // namespace tz
