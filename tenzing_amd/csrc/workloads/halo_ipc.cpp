// Halo workload, IPC transport: mapping the peers' grids, the collective preflight, kernel
// puts and copy-engine (SDMA) puts with arrival and credit counters, device-side waits, the
// counter reset after an aborted run, link probes. Relay routing: halo_relay.cpp; host split:
// halo_hostsplit.cpp.
#include "halo_internal.hpp"

namespace tz {

void HaloExchange::off_node_exchange(void *stream) const {
  // the directions that cross nodes, over RCCL (pack, shift, unpack; every rank issues the same
  // shifts in the same order): the IPC preflights run them beside their puts, so that the check
  // after an exchange covers every ghost cell
  const std::vector<int> far = off_node_dirs();
  if (far.empty()) return;
  TZ_CHECK(useRccl_, "directions that cross nodes need the RCCL transport");
  for (int i : far) pack(i, stream);
  for (int i : far) shift(i, stream);
  for (int i : far) unpack(opp_[i], stream);
}

void HaloExchange::ipc_preflight(Ctrl *ctrl) {
  // Complete exchanges through IPC before the search may use it: every ghost must arrive
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
  ipcTimeoutS_ = std::min(ipcTimeoutS_, preflight_wait_s());
  // two exchanges of different value generations (the caller's, then 2): the second must
  // deliver new data through the buffers (and past the caches) the first one used
  for (int gen = 1; gen <= 2 && bad == 0; ++gen) {
    if (gen > 1) {
      // my init_grid complete before anyone puts, theirs before my check
      init_grid(nullptr, gen);
      ctrl->barrier();
    }
    try {
      if (!local.empty()) direct_group(local, nullptr);
      off_node_exchange(nullptr); // (directions that cross nodes: RCCL, so the check is whole)
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
          why = "preflight exchange " + std::to_string(gen) + ": " + std::to_string(e) +
                " wait timeout(s), " + std::to_string(cells) + " wrong cells";
        }
      } catch (const std::exception &ex) {
        bad = 1;
        why = std::string("preflight check: ") + ex.what();
      }
    }
    ctrl->allreduce_max(&bad, 1);
  }
  ipcTimeoutS_ = keep;
  if (bad != 0) {
    ipcReady_ = false;
    ipcWhy_ = why.empty() ? "preflight failed on another rank" : why;
    TZ_LOG(Warn, "ipc transport disabled: " << ipcWhy_);
    TZ_CHECK(a_.transport != "ipc", "ipc transport requested but " << why);
  }
  init_grid();
}

void HaloExchange::copy_preflight(Ctrl *ctrl) {
  // The kernel-put preflight proves the mappings; the copy-engine puts take another path (the
  // runtime's peer copy, or the SDMA engines writing across the link), so each variant gets a
  // verified exchange of its own. A failure drops only that variant, on every rank.
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) local.push_back(i);
    else if (ipc_[i]) remote.push_back(i);
  }
  const std::string failEnv = std::getenv("TZ_FAIL_TRANSPORTS") ? std::getenv("TZ_FAIL_TRANSPORTS") : "";
  const char *names[2] = {"memcpy_put", "sdma_put"};
  const double keep = ipcTimeoutS_;
  ipcTimeoutS_ = std::min(ipcTimeoutS_, preflight_wait_s());
  for (int k = 0; k < 2; ++k) {
    double bad = 0;
    std::string why;
    // a generation the kernel-put preflight did not leave behind (it ended on 2, then 0)
    init_grid(nullptr, 3 - k);
    TZ_HIP(hipDeviceSynchronize());
    ctrl->barrier();
    try {
      if (!local.empty()) direct_group(local, nullptr);
      off_node_exchange(nullptr);
      copy_put_group(remote, nullptr, /*sdma=*/k == 1);
      wait_group(remote, nullptr);
      ipc_unpack_group(remote, nullptr);
      TZ_HIP(hipDeviceSynchronize());
    } catch (const std::exception &ex) {
      bad = 1;
      why = std::string(names[k]) + " preflight: " + ex.what();
    }
    ctrl->barrier(); // peers may still be copying into my receive buffers until they synced
    if (bad == 0) {
      try {
        const int e = ipc_errors();
        const uint64_t cells = check_grid();
        if (e || cells)
          why = std::string(names[k]) + " preflight: " + std::to_string(e) + " wait timeout(s), " +
                std::to_string(cells) + " wrong cells";
        else if (("," + failEnv + ",").find(std::string(",") + names[k] + ",") != std::string::npos)
          why = std::string(names[k]) + " preflight: simulated failure (TZ_FAIL_TRANSPORTS)";
        bad = why.empty() ? 0 : 1;
      } catch (const std::exception &ex) {
        bad = 1;
        why = std::string(names[k]) + " preflight check: " + ex.what();
      }
    }
    ctrl->allreduce_max(&bad, 1);
    if (bad != 0) {
      copyOk_[k] = false;
      copyWhy_[k] = why.empty() ? "preflight failed on another rank" : why;
      TZ_LOG(Warn, names[k] << " variant disabled: " << copyWhy_[k]);
      // a failed exchange leaves put / wait counters out of step: every rank resets them
      // together before the next variant's exchange
      reset_ipc_counters(ctrl);
    }
  }
  ipcTimeoutS_ = keep;
  useCopy_ = copyOk_[0] || copyOk_[1];
  init_grid();
}

bool HaloExchange::wide_puts_offered(const std::string &mode, const std::string &myBus,
                                     const std::vector<std::string> &peerBuses, int myDevice,
                                     const std::vector<int> &mappedDevices) {
  if (mode == "on") return true;
  if (mode != "auto") return false;
  for (const std::string &b : peerBuses)
    if (!b.empty() && !myBus.empty() && b != myBus) return true;
  for (int d : mappedDevices)
    if (d >= 0 && d != myDevice) return true;
  return false;
}

void HaloExchange::wide_put_preflight(Ctrl *ctrl) {
  // Offered or not, agreed first (the search needs the same graph on every rank): "auto" offers
  // the wide variant when any rank's peers live on another device, where the puts cross xGMI
  // links; ranks sharing one GPU store into their own HBM and gain nothing from it.
  // Which device a peer sits on: its PCI bus id (allgathered; every rank makes this call), and
  // the device the runtime reports for the peer memory mapped here (which may name the importing
  // device even for another GPU's memory, so the bus id decides as well).
  int dev = 0;
  TZ_HIP(hipGetDevice(&dev));
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, int(sizeof(bus)), dev) != hipSuccess) bus[0] = 0;
  const std::vector<std::string> buses = ctrl->allgather(std::string(bus));
  std::vector<std::string> peerBuses;
  for (int i = 0; i < ndirs(); ++i)
    if (ipc_[i] && size_t(nbr_[i]) < buses.size()) peerBuses.push_back(buses[size_t(nbr_[i])]);
  std::vector<int> mapped;
  for (const auto &[q, d] : ipc_peer_devices()) mapped.push_back(d);
  double offer = wide_puts_offered(a_.wide_puts, bus, peerBuses, dev, mapped) ? 1 : 0;
  ctrl->allreduce_max(&offer, 1);
  widePuts_ = false;
  if (offer == 0) return;
  if (a_.wide_put_blocks == kern::box_tuning().put_max_blocks) {
    wideWhy_ = "not offered: the same cap as the default put";
    return;
  }
  // then one verified exchange with the wide launches, like copy_preflight
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) local.push_back(i);
    else if (ipc_[i]) remote.push_back(i);
  }
  const double keep = ipcTimeoutS_;
  ipcTimeoutS_ = std::min(ipcTimeoutS_, preflight_wait_s());
  double bad = 0;
  std::string why;
  init_grid(nullptr, 3);
  TZ_HIP(hipDeviceSynchronize());
  ctrl->barrier();
  try {
    if (!local.empty()) direct_group(local, nullptr);
    off_node_exchange(nullptr);
    put_group(remote, nullptr, a_.wide_put_blocks);
    wait_group(remote, nullptr);
    if (!ipcGrid_) ipc_unpack_group(remote, nullptr);
    TZ_HIP(hipDeviceSynchronize());
  } catch (const std::exception &ex) {
    bad = 1;
    why = std::string("wide_put preflight: ") + ex.what();
  }
  ctrl->barrier(); // peers may still be putting into my ghosts until they synced
  if (bad == 0) {
    try {
      const int e = ipc_errors();
      const uint64_t cells = check_grid();
      if (e || cells)
        why = "wide_put preflight: " + std::to_string(e) + " wait timeout(s), " +
              std::to_string(cells) + " wrong cells";
      bad = why.empty() ? 0 : 1;
    } catch (const std::exception &ex) {
      bad = 1;
      why = std::string("wide_put preflight check: ") + ex.what();
    }
  }
  ctrl->allreduce_max(&bad, 1);
  ipcTimeoutS_ = keep;
  if (bad != 0) {
    wideWhy_ = why.empty() ? "preflight failed on another rank" : why;
    TZ_LOG(Warn, "wide_put variant disabled: " << wideWhy_);
    reset_ipc_counters(ctrl);
  } else {
    widePuts_ = true;
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
    // (relay routing adds four more sections: see kSlotSets)
    TZ_HIP(hipExtMallocWithFlags(&flags_, kSlotSets * nd * 8, hipDeviceMallocUncached));
    TZ_HIP(hipMemset(flags_, 0, kSlotSets * nd * 8));
    expected_ = DeviceBuffer(nd * 8);
    TZ_HIP(hipMemset(expected_.get(), 0, nd * 8));
    sent_ = DeviceBuffer(nd * 8);
    TZ_HIP(hipMemset(sent_.get(), 0, nd * 8));
    relayBook_ = DeviceBuffer(4 * nd * 8);
    TZ_HIP(hipMemset(relayBook_.get(), 0, relayBook_.bytes()));
    // block counters of signalling launches: one range per group keyed by its first direction,
    // in four sets (puts, relay corner puts, relay forwards, host-split host puts: these may
    // run beside each other)
    done_ = DeviceBuffer(4 * nd * kern::kMaxBoxes * sizeof(unsigned int));
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
    mine = node_identity() + handle_of(flags_);
    if (ipcGrid_) {
      mine += handle_of(grid());
    } else {
      for (int i = 0; i < ndirs(); ++i) mine += handle_of(ipc_[i] ? recv_[i].get() : nullptr);
      // relay routing: then the relay buffer of every direction ([flags][recv x nd][relay x nd])
      if (relay_)
        for (int i = 0; i < ndirs(); ++i)
          mine += handle_of(size_t(i) < relayBuf_.size() ? relayBuf_[i].get() : nullptr);
    }
    TZ_LOG(Info, "ipc: exported " << (ipcGrid_ ? "grid" : "receive buffers") << " and flags");
  } catch (const std::exception &e) {
    err = std::string("export: ") + e.what();
    mine.clear();
  }
  const std::vector<std::string> all = ctrl->allgather(mine);
  if (!err.empty()) return err;
  const std::string me = node_identity();
  auto open = [&](const std::string &blob, size_t k) {
    TZ_CHECK(blob.size() >= kNodeIdBytes + (k + 1) * H, "a peer exported no IPC handles");
    // a handle is only meaningful on the node that exported it
    TZ_CHECK(blob.compare(0, kNodeIdBytes, me) == 0, "a peer runs on another node");
    const char *at = blob.data() + kNodeIdBytes + k * H;
    hipIpcMemHandle_t h;
    std::memcpy(&h, at, H);
    TZ_CHECK(std::any_of(at, at + H, [](char c) { return c != 0; }),
             "a peer exported no IPC handle in slot " << k);
    void *p = nullptr;
    TZ_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(p);
    return p;
  };
  try {
    TZ_CHECK(int(all.size()) == a_.size, "allgather returned " << all.size() << " entries");
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
  if (relay_) {
    relayWhy_.clear();
    try {
      auto flags_of = [&](int q) {
        if (!peerFlags_[size_t(q)]) {
          TZ_LOG(Info, "ipc: mapping rank " << q << " (relay)");
          peerFlags_[size_t(q)] = open(all[size_t(q)], 0);
        }
      };
      peerRelay_.assign(nd, nullptr);
      peerFwdRecv_.assign(nd, nullptr);
      flags_of(corner_);
      flags_of(relayOrigin_);
      for (int i : relay_faces()) {
        flags_of(fwdTo_[i]);
        flags_of(fwdFrom_[i]);
        // my share relayed for direction i waits in the corner peer's relay buffer i; what I
        // forward for direction i goes to the final receiver's buffer of ghost side -d_i
        peerRelay_[size_t(i)] = open(all[size_t(corner_)], 1 + nd + size_t(i));
        peerFwdRecv_[size_t(i)] = open(all[size_t(fwdTo_[i])], 1 + size_t(opp_[i]));
      }
    } catch (const std::exception &e) {
      relayWhy_ = std::string("relay map: ") + e.what();
    }
  }
  return "";
}

std::map<int, int> HaloExchange::ipc_peer_devices() const {
  std::map<int, int> out;
  for (size_t q = 0; q < peerFlags_.size(); ++q) {
    if (!peerFlags_[q]) continue;
    hipPointerAttribute_t at{};
    out[int(q)] = hipPointerGetAttributes(&at, peerFlags_[q]) == hipSuccess ? at.device : -1;
  }
  return out;
}

void HaloExchange::put_group(const std::vector<int> &dirs, void *stream, int max_blocks) const {
  TZ_CHECK(ready() && ipcReady_, "ipc transport not set up");
  TZ_CHECK(!dirs.empty() && dirs.size() <= size_t(kern::kMaxBoxes), "bad put group");
  std::vector<kern::MoveDesc> ms;
  std::vector<kern::BoxDesc> bs;
  kern::MoveSignal sig;
  sig.max_blocks = max_blocks;
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

void HaloExchange::copy_put_group(const std::vector<int> &dirs, void *stream, bool sdma) const {
  // The copy-engine put: pack into my local send buffers (one launch), then one device-to-device
  // copy per direction into the receiver's IPC-mapped buffer, then one small kernel publishes
  // the arrivals. Same credit protocol as put_group. `sdma`: the copies are forced onto the SDMA
  // engines (hipMemcpyDeviceToDeviceNoCU), so the transfer takes no CUs at all; otherwise the
  // runtime picks the engine (hipMemcpyDeviceToDevice: blit kernels within one device, its
  // peer-copy path between devices). On loopback ranks (one GPU) the forced SDMA engines are
  // several times slower than the blit kernels (N=4: 0.49 ms vs 2.2 ms per exchange,
  // profiles/archive/r3_regress/), which is why both variants are offered and the search picks.
  TZ_CHECK(ready() && ipcReady_ && useCopy_ && !ipcGrid_, "ipc copy-engine puts not set up");
  TZ_CHECK(!dirs.empty() && dirs.size() <= size_t(kern::kMaxBoxes), "bad copy-put group");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<kern::BoxDesc> bs;
  std::vector<unsigned long long *> arrive;
  for (int i : dirs) {
    TZ_CHECK(i >= 0 && i < ndirs() && ipc_[i] && send_[i].get() && peerRecv_[size_t(i)],
             "direction " << i << " is not a copy-engine put");
    bs.push_back(pack_box(i)); // into my send buffer of direction i
    arrive.push_back(static_cast<unsigned long long *>(peerFlags_[size_t(nbr_[i])]) + i);
  }
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_) + ndirs(), sent_.as<unsigned long long>(),
                 dirs.data(), int(dirs.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/1);
  kern::box_copy_many(grid(), bs.data(), int(bs.size()), false, stream);
  std::vector<Copy> cs;
  for (int i : dirs) cs.push_back({peerRecv_[size_t(i)], send_[i].get(), box_elems(i) * sizeof(double)});
  engine_copies(cs, s, sdma);
  kern::ipc_signal(arrive.data(), int(arrive.size()), stream);
}

HaloExchange::EngineSet &HaloExchange::engines_for(void *stream) const {
  // one set of extra engine streams (and fork / join events) per schedule stream: two copy ops
  // on different schedule streams never share an engine queue, so neither waits for the other
  // (a hidden dependency the synchronizer and the race verifier could not see)
  std::lock_guard<std::mutex> lk(enginesMu_);
  EngineSet &e = engines_[stream];
  if (e.events.empty()) {
    // created lazily, possibly while `stream` is being captured: relaxed capture mode for the
    // creation calls, restored afterwards
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    TZ_HIP(hipThreadExchangeStreamCaptureMode(&mode));
    try {
      for (int k = 1; k < copyEngines_; ++k) {
        hipStream_t st = nullptr;
        TZ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        e.streams.push_back(st);
      }
      for (int k = 0; k < copyEngines_; ++k) {
        hipEvent_t ev = nullptr;
        TZ_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        e.events.push_back(ev);
      }
    } catch (...) {
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      throw;
    }
    TZ_HIP(hipThreadExchangeStreamCaptureMode(&mode));
  }
  return e;
}

void HaloExchange::engine_copies(const std::vector<Copy> &copies, void *stream, bool sdma) const {
  // Every copy is cut into one chunk per engine, chunk k on engine k: one SDMA engine cannot
  // fill an xGMI link, several can. Chunks are whole 256-B multiples so every engine moves
  // aligned spans. Engine 0 is the op's own stream; the others fork from it and join back,
  // which stream capture records as plain graph edges.
  hipStream_t s = static_cast<hipStream_t>(stream);
  const hipMemcpyKind kind = sdma ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
  auto copy = [kind](void *dst, const void *src, size_t n, hipStream_t st) {
    if (n) TZ_HIP(hipMemcpyAsync(dst, src, n, kind, st));
  };
  if (copyEngines_ <= 1) {
    for (const Copy &c : copies) copy(c.dst, c.src, c.bytes, s);
    return;
  }
  EngineSet &es = engines_for(stream);
  const int E = 1 + int(es.streams.size());
  hipEvent_t fork = static_cast<hipEvent_t>(es.events[0]);
  // fork: each engine stream starts behind exactly what `s` has enqueued so far. Inside a graph
  // capture, an engine stream already in the capture gets that dependency set replaced (a plain
  // event wait would ADD it to whatever the engine stream captured for an earlier op: a false
  // edge between independent copy ops that share the engine set of the capture stream)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long capId = 0;
  const hipGraphNode_t *dp = nullptr;
  size_t nd = 0;
  TZ_HIP(hipStreamGetCaptureInfo_v2(s, &cs, &capId, nullptr, &dp, &nd));
  std::vector<hipGraphNode_t> sDeps(dp, dp + nd);
  bool recorded = false;
  for (int k = 1; k < E; ++k) {
    hipStream_t e = static_cast<hipStream_t>(es.streams[size_t(k - 1)]);
    if (cs == hipStreamCaptureStatusActive) {
      hipStreamCaptureStatus ce = hipStreamCaptureStatusNone;
      unsigned long long eid = 0;
      TZ_HIP(hipStreamGetCaptureInfo_v2(e, &ce, &eid, nullptr, nullptr, nullptr));
      if (ce == hipStreamCaptureStatusActive && eid == capId) {
        TZ_HIP(hipStreamUpdateCaptureDependencies(e, sDeps.empty() ? nullptr : sDeps.data(), sDeps.size(),
                                                  hipStreamSetCaptureDependencies));
        continue;
      }
    }
    if (!recorded) {
      TZ_HIP(hipEventRecord(fork, s));
      recorded = true;
    }
    TZ_HIP(hipStreamWaitEvent(e, fork, 0));
  }
  for (const Copy &c : copies) {
    const size_t per = (c.bytes / size_t(E) + 255) / 256 * 256;
    for (int k = 0; k < E; ++k) {
      const size_t off = size_t(k) * per;
      if (off >= c.bytes) break;
      hipStream_t st = k == 0 ? s : static_cast<hipStream_t>(es.streams[size_t(k - 1)]);
      copy(static_cast<char *>(c.dst) + off, static_cast<const char *>(c.src) + off,
           std::min(per, c.bytes - off), st);
    }
  }
  for (int k = 1; k < E; ++k) {
    hipEvent_t join = static_cast<hipEvent_t>(es.events[size_t(k)]);
    TZ_HIP(hipEventRecord(join, static_cast<hipStream_t>(es.streams[size_t(k - 1)])));
    TZ_HIP(hipStreamWaitEvent(s, join, 0));
  }
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

void HaloExchange::reset_ipc_counters(Ctrl *ctrl) {
  // a half-done exchange leaves the counters out of step; with every rank idle (synchronized,
  // then a barrier) they all restart from zero, then a second barrier before anyone puts again
  try {
    TZ_HIP(hipDeviceSynchronize());
  } catch (const std::exception &) {
  }
  ctrl->barrier();
  TZ_HIP(hipMemset(flags_, 0, kSlotSets * size_t(ndirs()) * 8));
  TZ_HIP(hipMemset(expected_.get(), 0, expected_.bytes()));
  TZ_HIP(hipMemset(sent_.get(), 0, sent_.bytes()));
  TZ_HIP(hipMemset(relayBook_.get(), 0, relayBook_.bytes()));
  TZ_HIP(hipMemset(done_.get(), 0, done_.bytes()));
  TZ_HIP(hipMemset(err_.get(), 0, sizeof(int))); // the aborted waits' timeouts
  if (hsBook_.get()) TZ_HIP(hipMemset(hsBook_.get(), 0, hsBook_.bytes()));
  if (hsMine_.host()) std::memset(hsMine_.host(), 0, size_t(hsChunks_ + 1) * size_t(ndirs()) * 8);
  TZ_HIP(hipDeviceSynchronize());
  ctrl->barrier();
}

double HaloExchange::link_probe(int dir, const std::string &via, int iters, Ctrl *ctrl) {
  TZ_CHECK(ready() && ctrl && ctrl->size() == a_.size, "link probe needs a set-up exchange and its control plane");
  TZ_CHECK(dir >= 0 && dir < ndirs() && !direct_[dir], "direction " << dir << " is not remote");
  TZ_CHECK(iters >= 1, "iters must be positive");
  // "pair_put" / "pair_sdma" / "pair_mixed": both faces of the axis at once (one peer when the
  // dimension has 2 ranks), by kernel puts, copy engines, or one of each on two streams
  const bool pair = via.rfind("pair_", 0) == 0;
  const std::string how = pair ? via.substr(5) : via;
  // "put_wide": the kernel put with HaloArgs::wide_put_blocks workgroups per box; "put_cap<N>":
  // with N workgroups per box (a sweep of the put width over one link)
  const bool capped = how.rfind("put_cap", 0) == 0;
  const bool isPut = how == "put" || how == "put_wide" || capped;
  int cap = how == "put_wide" ? a_.wide_put_blocks : 0;
  if (capped) {
    cap = std::atoi(how.c_str() + 7);
    TZ_CHECK(cap >= 1 && cap <= 4096, "put_cap<N> needs 1 <= N <= 4096 (got " << how << ")");
  }
  const std::vector<int> d = pair ? std::vector<int>{dir, opp_[dir]} : std::vector<int>{dir};
  hipStream_t s = nullptr, s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto release = [&] { // also on error paths: the first failure is the one reported
    if (s2) (void)hipStreamDestroy(s2);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    (void)hipStreamDestroy(s);
  };
  if (how == "mixed") {
    TZ_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    TZ_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    TZ_HIP(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  }
  auto once = [&] {
    if (pair && (isPut || how == "sdma" || how == "mixed")) {
      TZ_CHECK(ipcReady_ && ipc_[d[0]] && ipc_[d[1]], "ipc transport not available");
      if (isPut) {
        put_group(d, s, cap);
      } else if (how == "sdma") {
        copy_put_group(d, s);
      } else { // + face by CU stores on s, - face by the copy engines on s2, concurrently
        TZ_HIP(hipEventRecord(fork, s));
        TZ_HIP(hipStreamWaitEvent(s2, fork, 0));
        put_group({d[0]}, s);
        copy_put_group({d[1]}, s2);
        TZ_HIP(hipEventRecord(join, s2));
        TZ_HIP(hipStreamWaitEvent(s, join, 0));
      }
      wait_group(d, s);
      if (!ipcGrid_) ipc_unpack_group(d, s);
    } else if (pair) {
      TZ_THROW("pair probes take put, put_wide, sdma or mixed (got " << how << ")");
    } else if (isPut || via == "sdma" || via == "memcpy") {
      TZ_CHECK(ipcReady_ && ipc_[dir], "ipc transport not available");
      if (isPut) put_group(d, s, cap);
      else copy_put_group(d, s, via == "sdma");
      wait_group(d, s);
      if (!ipcGrid_) ipc_unpack_group(d, s);
    } else if (via == "rccl") {
      TZ_CHECK(useRccl_ && pipe_[dir], "RCCL transport not available");
      pack_group(d, s);
      shift_group(d, s, 0);
      unpack_group(d, s);
    } else {
      TZ_THROW("link probe transport must be put, put_wide, sdma, memcpy or rccl (got " << via << ")");
    }
  };
  // agree collectively that every rank can run the probe before any transfer is issued
  std::string err;
  const bool ipcOk = ipcReady_ && ipc_[dir] && (!pair || ipc_[opp_[dir]]);
  if ((isPut || how == "sdma" || how == "mixed") && !(ipcOk && (isPut || (useCopy_ && !ipcGrid_))))
    err = via + " unavailable";
  if (via == "rccl" && !(useRccl_ && pipe_[dir])) err = "rccl unavailable";
  double bad = err.empty() ? 0.0 : 1.0;
  ctrl->allreduce_max(&bad, 1);
  if (bad != 0) {
    release();
    TZ_THROW("link probe: " << (err.empty() ? via + " unavailable on another rank" : err));
  }
  // a local failure travels with the collectives (every rank makes the same calls), so all
  // ranks throw together instead of leaving peers in a barrier
  auto agree = [&](std::string &e, double *v) {
    double red[2] = {v ? *v : 0.0, e.empty() ? 0.0 : 1.0};
    ctrl->allreduce_max(red, 2);
    if (v) *v = red[0];
    if (red[1] != 0.0) {
      (void)hipStreamSynchronize(s);
      if (s2) (void)hipStreamSynchronize(s2);
      release();
      TZ_THROW("link probe (" << via << ") failed" << (e.empty() ? " on another rank" : ": " + e));
    }
  };
  std::string e;
  try {
    once(); // warm-up (first-use mappings, RCCL connections)
    TZ_HIP(hipStreamSynchronize(s));
  } catch (const std::exception &x) {
    e = x.what();
  }
  agree(e, nullptr);
  double t = 0;
  try {
    const double t0 = wtime();
    for (int k = 0; k < iters; ++k) once();
    TZ_HIP(hipStreamSynchronize(s));
    t = (wtime() - t0) / iters;
  } catch (const std::exception &x) {
    e = x.what();
  }
  agree(e, &t); // (also: peers may write into my buffers until every rank got here)
  release();
  return t;
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
