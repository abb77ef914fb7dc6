// Halo workload, IPC transport: mapping the peers' grids, the collective preflight, kernel
// puts and copy-engine (SDMA) puts with arrival and credit counters, device-side waits.
#include "halo_internal.hpp"

namespace tz {

void HaloExchange::ipc_preflight(Ctrl *ctrl) {
  // One complete exchange through IPC before the search may use it: every ghost must arrive
  // (no wait timeout) and be right on every rank. A mapping that "works" but does not deliver
  // (or delivers wrong data) turns the transport off collectively instead of costing a wait
  // timeout per iteration of every IPC candidate later.
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) local.push_back(i);
    else if (ipc_[i]) remote.push_back(i);
  }
  double bad = 0;
  std::string why;
  const double keep = ipcTimeoutS_;
  ipcTimeoutS_ = std::min(ipcTimeoutS_, 3.0);
  try {
    if (!local.empty()) direct_group(local, nullptr);
    put_group(remote, nullptr);
    wait_group(remote, nullptr);
    if (!ipcGrid_) ipc_unpack_group(remote, nullptr);
    TZ_HIP(hipDeviceSynchronize());
  } catch (const std::exception &ex) {
    bad = 1;
    why = std::string("preflight exchange: ") + ex.what();
  }
  // peers may still be putting into my ghosts until they have synchronized too (outside the
  // try: every rank reaches this collective whatever failed locally)
  ctrl->barrier();
  if (bad == 0) {
    try {
      const int e = ipc_errors();
      const uint64_t cells = check_grid();
      if (e || cells) {
        bad = 1;
        why = "preflight exchange: " + std::to_string(e) + " wait timeout(s), " +
              std::to_string(cells) + " wrong cells";
      }
    } catch (const std::exception &ex) {
      bad = 1;
      why = std::string("preflight check: ") + ex.what();
    }
  }
  ipcTimeoutS_ = keep;
  ctrl->allreduce_max(&bad, 1);
  if (bad != 0) {
    ipcReady_ = false;
    TZ_LOG(Warn, "ipc transport disabled: " << (why.empty() ? "failed on another rank" : why));
    TZ_CHECK(a_.transport != "ipc", "ipc transport requested but " << why);
  }
  init_grid();
}

std::string HaloExchange::setup_ipc(Ctrl *ctrl) {
  // Collective: every rank makes the same control-plane calls (one allgather) whatever fails
  // locally, and reports failure as a string, so a rank that cannot export or map never leaves
  // the others blocked in a mismatched collective.
  TZ_CHECK(ctrl && ctrl->size() == a_.size, "ipc transport needs a control plane of size " << a_.size);
  if (const char *v = std::getenv("TZ_IPC_TIMEOUT")) ipcTimeoutS_ = std::atof(v);
  const size_t nd = size_t(ndirs());
  const size_t H = sizeof(hipIpcMemHandle_t);
  std::string mine, err;
  try {
    // arrival counters live in uncached memory: a remote GPU's system-scope atomics land in
    // HBM and the local spin loads (system scope) see them without stale cache lines
    // [arrivals of direction i | credits of direction i]: a receiver counts the puts it got in
    // slot i and, once it has consumed them, returns a credit to the sender's slot nd + i
    TZ_HIP(hipExtMallocWithFlags(&flags_, std::max<size_t>(2 * nd * 8, 64), hipDeviceMallocUncached));
    TZ_HIP(hipMemset(flags_, 0, 2 * nd * 8));
    expected_ = DeviceBuffer(nd * 8);
    TZ_HIP(hipMemset(expected_.get(), 0, nd * 8));
    sent_ = DeviceBuffer(nd * 8);
    TZ_HIP(hipMemset(sent_.get(), 0, nd * 8));
    done_ = DeviceBuffer(nd * kern::kMaxBoxes * sizeof(unsigned int));
    TZ_HIP(hipMemset(done_.get(), 0, done_.bytes()));
    err_ = DeviceBuffer(sizeof(int));
    TZ_HIP(hipMemset(err_.get(), 0, sizeof(int)));
    TZ_HIP(hipDeviceSynchronize());
    // exported: [flags][grid] ("grid" mode) or [flags][recv buffer of every direction]
    auto handle_of = [&](void *p) {
      hipIpcMemHandle_t h;
      std::memset(&h, 0, sizeof(h));
      if (p) TZ_HIP(hipIpcGetMemHandle(&h, p));
      return std::string(reinterpret_cast<const char *>(&h), H);
    };
    mine = handle_of(flags_);
    if (ipcGrid_) {
      mine += handle_of(grid());
    } else {
      for (int i = 0; i < ndirs(); ++i) mine += handle_of(ipc_[i] ? recv_[i].get() : nullptr);
    }
    TZ_LOG(Info, "ipc: exported " << (ipcGrid_ ? "grid" : "receive buffers") << " and flags");
  } catch (const std::exception &e) {
    err = std::string("export: ") + e.what();
    mine.clear();
  }
  const std::vector<std::string> all = ctrl->allgather(mine);
  if (!err.empty()) return err;
  try {
    TZ_CHECK(int(all.size()) == a_.size, "allgather returned " << all.size() << " entries");
    auto open = [&](const std::string &blob, size_t k) {
      TZ_CHECK(blob.size() >= (k + 1) * H, "a peer exported no IPC handles");
      hipIpcMemHandle_t h;
      std::memcpy(&h, blob.data() + k * H, H);
      void *p = nullptr;
      TZ_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(p);
      return p;
    };
    peerGrid_.assign(size_t(a_.size), nullptr);
    peerFlags_.assign(size_t(a_.size), nullptr);
    peerRecv_.assign(nd, nullptr);
    for (int i = 0; i < ndirs(); ++i) {
      if (!ipc_[i]) continue;
      const int q = nbr_[i];
      const std::string &blob = all[size_t(q)];
      if (!peerFlags_[size_t(q)]) {
        TZ_LOG(Info, "ipc: mapping rank " << q);
        peerFlags_[size_t(q)] = open(blob, 0);
        if (ipcGrid_) peerGrid_[size_t(q)] = open(blob, 1);
      }
      // my slab facing d_i fills q's ghost side -d_i, staged in q's recv buffer of that side
      if (!ipcGrid_) peerRecv_[size_t(i)] = open(blob, 1 + size_t(opp_[i]));
    }
  } catch (const std::exception &e) {
    return std::string("map: ") + e.what();
  }
  return "";
}

void HaloExchange::put_group(const std::vector<int> &dirs, void *stream) const {
  TZ_CHECK(ready() && ipcReady_, "ipc transport not set up");
  TZ_CHECK(!dirs.empty() && dirs.size() <= size_t(kern::kMaxBoxes), "bad put group");
  std::vector<kern::MoveDesc> ms;
  std::vector<kern::BoxDesc> bs;
  kern::MoveSignal sig;
  // block counters: one slot range per group, keyed by its first direction (groups of one
  // schedule are disjoint, so concurrently running puts never share counters)
  sig.done = done_.as<unsigned int>() + size_t(dirs.front()) * kern::kMaxBoxes;
  // flow control: put n+1 of direction i may only overwrite the peer's ghosts / receive buffer
  // after the peer has consumed put n (its credit, returned to my slot nd + i)
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_) + ndirs(), sent_.as<unsigned long long>(),
                 dirs.data(), int(dirs.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/1);
  for (size_t k = 0; k < dirs.size(); ++k) {
    const int i = dirs[k];
    TZ_CHECK(i >= 0 && i < ndirs() && ipc_[i], "direction " << i << " is not an ipc put");
    const int q = nbr_[i];
    // the receiver counts arrivals of direction i in its slot i
    sig.flag[k] = static_cast<unsigned long long *>(peerFlags_[size_t(q)]) + i;
    if (!ipcGrid_) {
      kern::BoxDesc b = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
      b.buf = static_cast<double *>(peerRecv_[size_t(i)]);
      bs.push_back(b);
      continue;
    }
    const kern::BoxDesc s = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
    const kern::BoxDesc d = make_box(a_, dirs_[opp_[i]], true, xoff_, sy_, sz_, sq_);
    kern::MoveDesc m;
    m.src = grid();
    m.dst = static_cast<double *>(peerGrid_[size_t(q)]);
    m.src_off = s.grid_off;
    m.dst_off = d.grid_off;
    m.s1 = s.s1;
    m.s2 = s.s2;
    m.s3 = s.s3;
    m.len = s.len;
    m.n1 = s.n1;
    m.n2 = s.n2;
    m.n3 = s.n3;
    ms.push_back(m);
  }
  if (ipcGrid_) kern::box_move_many_signal(ms.data(), int(ms.size()), sig, stream);
  else kern::box_pack_many_signal(grid(), bs.data(), int(bs.size()), sig, stream);
}

void HaloExchange::copy_put_group(const std::vector<int> &dirs, void *stream) const {
  // The copy-engine put: pack into my local send buffers (one launch), then one device-to-device
  // copy per direction into the receiver's IPC-mapped buffer. Across GPUs HIP runs these on the
  // SDMA engines, so the xGMI transfer itself takes no CUs (they stay free for concurrent local
  // work); then one small kernel publishes the arrivals. Same credit protocol as put_group.
  TZ_CHECK(ready() && ipcReady_ && useCopy_ && !ipcGrid_, "ipc copy-engine puts not set up");
  TZ_CHECK(!dirs.empty() && dirs.size() <= size_t(kern::kMaxBoxes), "bad copy-put group");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<kern::BoxDesc> bs;
  std::vector<unsigned long long *> arrive;
  for (int i : dirs) {
    TZ_CHECK(i >= 0 && i < ndirs() && ipc_[i] && send_[i].get() && peerRecv_[size_t(i)],
             "direction " << i << " is not a copy-engine put");
    kern::BoxDesc b = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
    b.buf = send_[i].as<double>();
    bs.push_back(b);
    arrive.push_back(static_cast<unsigned long long *>(peerFlags_[size_t(nbr_[i])]) + i);
  }
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_) + ndirs(), sent_.as<unsigned long long>(),
                 dirs.data(), int(dirs.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/1);
  kern::box_copy_many(grid(), bs.data(), int(bs.size()), false, stream);
  for (int i : dirs)
    TZ_HIP(hipMemcpyAsync(peerRecv_[size_t(i)], send_[i].get(), box_elems(i) * sizeof(double),
                          hipMemcpyDeviceToDevice, s));
  kern::ipc_signal(arrive.data(), int(arrive.size()), stream);
}

void HaloExchange::wait_group(const std::vector<int> &dirs, void *stream) const {
  TZ_CHECK(ready() && ipcReady_, "ipc transport not set up");
  for (int i : dirs) TZ_CHECK(i >= 0 && i < ndirs() && ipc_[i], "direction " << i << " is not an ipc put");
  // grid mode: the ghosts are consumed once they arrived (nothing reads them inside the
  // exchange), so the credit goes back right after the wait; buffers mode returns it after
  // the unpack (ipc_unpack_group)
  const std::vector<unsigned long long *> credits = credit_ptrs(dirs);
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_), expected_.as<unsigned long long>(),
                 dirs.data(), int(dirs.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/0,
                 ipcGrid_ ? credits.data() : nullptr);
}

std::vector<unsigned long long *> HaloExchange::credit_ptrs(const std::vector<int> &dirs) const {
  // the put that filled my slot i came from nbr(-i); its credit slot for direction i is nd + i
  std::vector<unsigned long long *> v;
  for (int i : dirs) {
    const int from = nbr_[opp_[i]];
    TZ_CHECK(peerFlags_.size() > size_t(from) && peerFlags_[size_t(from)],
             "rank " << from << " is not IPC-mapped");
    v.push_back(static_cast<unsigned long long *>(peerFlags_[size_t(from)]) + ndirs() + i);
  }
  return v;
}

void HaloExchange::ipc_unpack_group(const std::vector<int> &dirs, void *stream) const {
  TZ_CHECK(ready() && ipcReady_ && !ipcGrid_, "ipc buffers mode not set up");
  unpack_group(dirs, stream);
  const std::vector<unsigned long long *> credits = credit_ptrs(dirs);
  kern::ipc_signal(credits.data(), int(credits.size()), stream);
}

int HaloExchange::ipc_errors() {
  if (!useIpc_ || !err_.get()) return 0;
  int e = 0;
  TZ_HIP(hipDeviceSynchronize());
  err_.download(&e, sizeof(e));
  TZ_HIP(hipMemset(err_.get(), 0, sizeof(int)));
  return e;
}

} // namespace tz
