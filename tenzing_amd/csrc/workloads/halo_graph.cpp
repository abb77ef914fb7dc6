// Halo workload, op graph: the GPU ops and the graph builder with its ChoiceOps (per-direction
// or fused groups, RCCL / IPC / SDMA transport, stencil placement).
// Reference: src/halo_exchange/ops_halo_exchange.cu:33-84 (HaloExchange::add_to_graph).
#include "halo_internal.hpp"

namespace tz {

namespace {

// byte-cost model for the simulator: ~5 TB/s effective HBM stream + launch latency
double copy_cost_us(double bytes) { return 3.0 + bytes / 5.0e6; }

// link-aware model (SimParams::link_model): the bytes of `dirs` (times `scale`) to each peer,
// one transfer per peer by `engine`; `hbm`: plus the local reads of them
std::vector<Traffic> to_peers(const HaloExchange &h, const std::vector<int> &dirs, const std::string &engine,
                              double scale = 1.0, bool hbm = true) {
  std::map<int, double> per;
  double total = 0;
  for (int i : dirs) {
    const double b = scale * 8.0 * double(h.box_elems(i));
    per[h.neighbor(i)] += b;
    total += b;
  }
  std::vector<Traffic> t;
  for (const auto &kv : per) t.push_back({"xgmi:" + std::to_string(kv.first), engine, kv.second});
  if (hbm && total > 0) t.push_back({"hbm", "kernel", total});
  return t;
}
std::vector<Traffic> local_hbm(double bytes) { return {{"hbm", "kernel", bytes}}; }
double dirs_bytes(const HaloExchange &h, const std::vector<int> &dirs) {
  double b = 0;
  for (int i : dirs) b += 8.0 * double(h.box_elems(i));
  return b;
}

// relay routing (2x2x2): the corner peer (all three axes differ) and the edge peers (two differ)
int corner_peer(const HaloExchange &h) {
  for (int i = 0; i < h.ndirs(); ++i) {
    const auto d = h.dir(i);
    if (d.dx && d.dy && d.dz) return h.neighbor(i);
  }
  return -1;
}
std::vector<int> edge_peers(const HaloExchange &h) {
  std::vector<int> v;
  for (int i = 0; i < h.ndirs(); ++i) {
    const auto d = h.dir(i);
    if ((d.dx != 0) + (d.dy != 0) + (d.dz != 0) == 2 &&
        std::find(v.begin(), v.end(), h.neighbor(i)) == v.end())
      v.push_back(h.neighbor(i));
  }
  return v;
}
// the direct part of a relayed / host-split exchange: (1 - frac) of every face, all the rest
std::vector<Traffic> split_direct(const HaloExchange &h, const std::vector<int> &dirs,
                                  const std::vector<int> &faces, double frac) {
  std::vector<int> f, rest;
  for (int i : dirs) (std::find(faces.begin(), faces.end(), i) != faces.end() ? f : rest).push_back(i);
  std::vector<Traffic> t = to_peers(h, f, "put", 1.0 - frac);
  for (const Traffic &x : to_peers(h, rest, "put")) t.push_back(x);
  return t;
}

class HaloPack : public GpuOp {
public:
  HaloPack(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_pack_" + h_->dir(i_).name(); }
  std::string kind() const override { return "HaloPack"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  double cost_us() const override { return copy_cost_us(bytes()); }
  std::vector<Traffic> traffic() const override { return local_hbm(bytes()); }
  void launch(void *s, Executor &) const override { h_->pack(i_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
};

class HaloUnpack : public GpuOp {
public:
  HaloUnpack(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_unpack_" + h_->dir(i_).name(); }
  std::string kind() const override { return "HaloUnpack"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  double cost_us() const override { return copy_cost_us(bytes()); }
  std::vector<Traffic> traffic() const override { return local_hbm(bytes()); }
  void launch(void *s, Executor &) const override { h_->unpack(i_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
};

class HaloShift : public GpuOp {
public:
  HaloShift(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_shift_" + h_->dir(i_).name(); }
  std::string kind() const override { return h_->uses_rccl() ? "HaloShift" : "HaloCopy"; }
  double bytes() const override { return 8.0 * double(h_->box_elems(i_)); }
  // xGMI link ~100 GB/s effective per direction + RCCL launch; self copy ~2.5 TB/s
  double cost_us() const override {
    return h_->uses_rccl() ? 8.0 + bytes() / 1.0e5 : 3.0 + bytes() / 2.5e6;
  }
  std::string order_domain() const override { return h_->uses_rccl() ? "rccl" : ""; }
  // RCCL inside hipGraphs only once the preflight verified it (else the runtime runs eagerly)
  bool capturable() const override { return !h_->uses_rccl() || h_->rccl_graph_ok(); }
  std::vector<Traffic> traffic() const override {
    if (!h_->uses_rccl()) return local_hbm(2.0 * bytes());
    std::vector<Traffic> t = to_peers(*h_, {i_}, "rccl", 1.0, false);
    t.push_back({"hbm", "kernel", 2.0 * bytes()}); // send buffer read, receive buffer written
    return t;
  }
  double latency_us() const override { return h_->uses_rccl() ? 8.0 : 3.0; }
  void launch(void *s, Executor &ex) const override { h_->shift(i_, s, ex.stream_index(s)); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
};

/// direct transport of one direction: interior slab -> neighbour's ghost (no buffers)
class HaloDirect : public GpuOp {
public:
  HaloDirect(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_direct_" + h_->dir(i_).name(); }
  std::string kind() const override { return "HaloDirect"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  double cost_us() const override { return copy_cost_us(bytes()); }
  std::vector<Traffic> traffic() const override { return local_hbm(bytes()); }
  double latency_us() const override { return 3.0; }
  void launch(void *s, Executor &) const override { h_->direct(i_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
};

/// ipc transport: pack-free put of one direction into the neighbour's grid + arrival signal
/// (`cap` > 0: a wide put, at most `cap` workgroups per box)
class HaloPut : public GpuOp {
public:
  HaloPut(std::shared_ptr<const HaloExchange> h, int i, int cap = 0) : h_(std::move(h)), i_(i), cap_(cap) {}
  std::string name() const override { return (cap_ ? "he_putw_" : "he_put_") + h_->dir(i_).name(); }
  std::string kind() const override { return cap_ ? "HaloWidePut" : "HaloPut"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  // peer stores over one xGMI link (~60 GB/s effective)
  double cost_us() const override { return 4.0 + bytes() / 2.0 / 6.0e4; }
  std::vector<Traffic> traffic() const override { return to_peers(*h_, {i_}, cap_ ? "wide" : "put"); }
  void launch(void *s, Executor &) const override { h_->put_group({i_}, s, cap_); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_, cap_;
};

/// stencil over an interior region (stencil mode)
class HaloStencil : public GpuOp {
public:
  HaloStencil(std::shared_ptr<const HaloExchange> h, int region) : h_(std::move(h)), region_(region) {}
  std::string name() const override {
    static const char *n[] = {"st_interior", "st_boundary", "st_full"};
    return n[region_];
  }
  std::string kind() const override { return "Stencil7"; }
  double bytes() const override {
    const auto &a = h_->args();
    const double n3 = double(a.nx) * a.ny * a.nz, in3 = double(a.nx - 2) * (a.ny - 2) * (a.nz - 2);
    const double cells = region_ == 0 ? in3 : (region_ == 1 ? n3 - in3 : n3);
    return 16.0 * cells * a.nq;
  }
  double cost_us() const override { return 3.0 + bytes() / 4.0e6; }
  std::vector<Traffic> traffic() const override { return local_hbm(bytes()); }
  void launch(void *s, Executor &) const override { h_->stencil(region_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int region_;
};

/// ipc transport: device-side wait for the neighbours' puts into my ghosts
class HaloWait : public GpuOp {
public:
  HaloWait(std::shared_ptr<const HaloExchange> h, std::vector<int> dirs, std::string tag)
      : h_(std::move(h)), dirs_(std::move(dirs)), tag_(std::move(tag)) {}
  std::string name() const override { return "he_wait_" + tag_; }
  std::string kind() const override { return "HaloWait"; }
  double cost_us() const override { return 3.0; }
  void launch(void *s, Executor &) const override { h_->wait_group(dirs_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  std::vector<int> dirs_;
  std::string tag_;
};

/// one op for a whole group of directions (single kernel launch / single RCCL group)
class HaloStageGroup : public GpuOp {
public:
  // UnpackRelease: unpack IPC receive buffers, then hand them back to the senders (credits)
  // CopyPut: pack locally, copy-engine (SDMA) copy into the peer's receive buffer, signal
  // MemcpyPut: the same with the runtime's choice of copy engine (hipMemcpyDeviceToDevice)
  // WidePut: Put with at most `cap` workgroups per box (HaloArgs::wide_puts)
  enum Stage { Pack, Shift, Unpack, Direct, Put, UnpackRelease, CopyPut, MemcpyPut, WidePut };
  HaloStageGroup(std::shared_ptr<const HaloExchange> h, Stage st, std::vector<int> dirs, std::string tag,
                 int cap = 0)
      : h_(std::move(h)), st_(st), dirs_(std::move(dirs)), tag_(std::move(tag)), cap_(cap) {}
  std::string name() const override {
    static const char *pre[] = {"he_pack_", "he_shift_", "he_unpack_", "he_direct_", "he_put_",
                                "he_unpack_", "he_copyput_", "he_mcput_", "he_putw_"};
    return pre[st_] + tag_;
  }
  std::string kind() const override {
    static const char *k[] = {"HaloPackGroup", "HaloShiftGroup", "HaloUnpackGroup",
                              "HaloDirectGroup", "HaloPutGroup", "HaloUnpackGroup",
                              "HaloCopyPutGroup", "HaloMemcpyPutGroup", "HaloWidePutGroup"};
    return k[st_];
  }
  double bytes() const override {
    double b = 0;
    for (int i : dirs_) b += 8.0 * double(h_->box_elems(i));
    return (st_ == Shift ? 1.0 : 2.0) * b;
  }
  double cost_us() const override {
    if (st_ == Shift) return h_->uses_rccl() ? 10.0 + bytes() / 3.0e5 : 3.0 + bytes() / 2.5e6;
    return copy_cost_us(bytes());
  }
  std::string order_domain() const override { return st_ == Shift && h_->uses_rccl() ? "rccl" : ""; }
  bool capturable() const override { return !(st_ == Shift && h_->uses_rccl()) || h_->rccl_graph_ok(); }
  std::vector<Traffic> traffic() const override {
    switch (st_) {
    case Shift:
      if (!h_->uses_rccl()) return local_hbm(2.0 * bytes());
      {
        std::vector<Traffic> t = to_peers(*h_, dirs_, "rccl", 1.0, false);
        t.push_back({"hbm", "kernel", 2.0 * bytes()});
        return t;
      }
    case Put: return to_peers(*h_, dirs_, "put");
    case WidePut: return to_peers(*h_, dirs_, "wide");
    case CopyPut:
    case MemcpyPut: {
      // pack locally (read + write), then the copy engines move the buffer to each peer
      std::vector<Traffic> t = to_peers(*h_, dirs_, st_ == CopyPut ? "sdma" : "memcpy", 1.0, false);
      t.push_back({"hbm", "kernel", bytes()});
      return t;
    }
    default: return local_hbm(bytes());
    }
  }
  double latency_us() const override { return st_ == Shift && h_->uses_rccl() ? 10.0 : 4.0; }
  void launch(void *s, Executor &ex) const override {
    if (st_ == Pack) h_->pack_group(dirs_, s);
    else if (st_ == Shift) h_->shift_group(dirs_, s, ex.stream_index(s));
    else if (st_ == Unpack) h_->unpack_group(dirs_, s);
    else if (st_ == Direct) h_->direct_group(dirs_, s);
    else if (st_ == Put) h_->put_group(dirs_, s);
    else if (st_ == WidePut) h_->put_group(dirs_, s, cap_);
    else if (st_ == CopyPut) h_->copy_put_group(dirs_, s, /*sdma=*/true);
    else if (st_ == MemcpyPut) h_->copy_put_group(dirs_, s, /*sdma=*/false);
    else h_->ipc_unpack_group(dirs_, s);
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  Stage st_;
  std::vector<int> dirs_;
  std::string tag_;
  int cap_;
};

/// relay routing stages (HaloArgs::relay): one op each, for every direction at once
class HaloRelay : public GpuOp {
public:
  enum Stage { PutDirect, PutCorner, Forward, Wait, Unpack, ForwardCopy };
  HaloRelay(std::shared_ptr<const HaloExchange> h, Stage st, std::vector<int> dirs, double frac)
      : h_(std::move(h)), st_(st), dirs_(std::move(dirs)), faces_(h_->relay_faces()), frac_(frac) {}
  std::string name() const override {
    static const char *post[] = {"putd", "putc", "fwd", "wait", "unpack", "fwdcp"};
    return "he_rl" + std::to_string(int(std::lround(frac_ * 100))) + "_" + post[st_];
  }
  std::string kind() const override {
    static const char *k[] = {"HaloRelayPutDirect", "HaloRelayPutCorner", "HaloRelayForward",
                              "HaloRelayWait", "HaloRelayUnpack", "HaloRelayForwardCopy"};
    return k[st_];
  }
  double bytes() const override {
    double faces = 0, rest = 0;
    for (int i : dirs_) {
      const bool face = std::find(faces_.begin(), faces_.end(), i) != faces_.end();
      (face ? faces : rest) += 8.0 * double(h_->box_elems(i));
    }
    if (st_ == PutDirect) return (1.0 - frac_) * faces + rest;
    if (st_ == PutCorner || st_ == Forward || st_ == ForwardCopy) return frac_ * faces;
    return st_ == Unpack ? 2.0 * (faces + rest) : 0.0;
  }
  // puts and forwards cross xGMI links (~60 GB/s effective each): the direct put uses the 3
  // face links at once, the corner put one link, a forward 3 edge links
  double cost_us() const override {
    if (st_ == Wait) return 3.0;
    if (st_ == Unpack) return copy_cost_us(bytes());
    const double links = st_ == PutCorner ? 1.0 : 3.0;
    return 4.0 + bytes() / links / 6.0e4;
  }
  std::vector<Traffic> traffic() const override {
    const double shared = frac_ * dirs_bytes(*h_, faces_);
    switch (st_) {
    case PutDirect: return split_direct(*h_, dirs_, faces_, frac_);
    case PutCorner: {
      const int c = corner_peer(*h_);
      return {{"xgmi:" + std::to_string(c), "put", shared}, {"hbm", "kernel", shared}};
    }
    case Forward:
    case ForwardCopy: {
      // as the corner of other ranks: their shares on to their face neighbours, my edge peers
      const std::vector<int> e = edge_peers(*h_);
      std::vector<Traffic> t;
      for (int q : e)
        t.push_back({"xgmi:" + std::to_string(q), st_ == Forward ? "put" : "sdma", shared / double(e.size())});
      t.push_back({"hbm", "kernel", shared});
      return t;
    }
    case Unpack: return local_hbm(bytes());
    default: return {};
    }
  }
  void launch(void *s, Executor &) const override {
    switch (st_) {
    case PutDirect: h_->relay_put_direct(dirs_, frac_, s); break;
    case PutCorner: h_->relay_put_corner(faces_, frac_, s); break;
    case Forward: h_->relay_forward(faces_, frac_, s); break;
    case ForwardCopy: h_->relay_forward(faces_, frac_, s, /*sdma=*/true); break;
    case Wait: h_->relay_wait(dirs_, faces_, s); break;
    case Unpack: h_->relay_unpack(dirs_, faces_, frac_, s); break;
    }
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  Stage st_;
  std::vector<int> dirs_, faces_;
  double frac_;
};

/// host split stages (HaloArgs::hostsplit): one op each, for every direction at once
class HaloHostSplit : public GpuOp {
public:
  enum Stage { PutDirect, PutHost, Wait, Unpack };
  HaloHostSplit(std::shared_ptr<const HaloExchange> h, Stage st, std::vector<int> dirs, double frac)
      : h_(std::move(h)), st_(st), dirs_(std::move(dirs)), faces_(h_->relay_faces()), frac_(frac) {}
  std::string name() const override {
    static const char *post[] = {"putd", "puth", "wait", "unpack"};
    return "he_hs" + std::to_string(int(std::lround(frac_ * 100))) + "_" + post[st_];
  }
  std::string kind() const override {
    static const char *k[] = {"HaloSplitPutDirect", "HaloSplitPutHost", "HaloSplitWait",
                              "HaloSplitUnpack"};
    return k[st_];
  }
  double bytes() const override {
    double faces = 0, rest = 0;
    for (int i : dirs_) {
      const bool face = std::find(faces_.begin(), faces_.end(), i) != faces_.end();
      (face ? faces : rest) += 8.0 * double(h_->box_elems(i));
    }
    if (st_ == PutDirect) return (1.0 - frac_) * faces + rest;
    if (st_ == PutHost) return frac_ * faces;
    return st_ == Unpack ? 2.0 * (faces + rest) : 0.0;
  }
  // xGMI face links ~60 GB/s effective each (3 at once); the host share crosses this GPU's
  // PCIe link (~40 GB/s) into host memory, and the receiver's, by DMA, back out
  double cost_us() const override {
    if (st_ == Wait) return 3.0;
    if (st_ == Unpack) return copy_cost_us(bytes()) + frac_ * 2.0 * bytes() / 4.0e4;
    return 4.0 + bytes() / (st_ == PutHost ? 4.0e4 : 3.0 * 6.0e4);
  }
  std::vector<Traffic> traffic() const override {
    const double shared = frac_ * dirs_bytes(*h_, faces_);
    switch (st_) {
    case PutDirect: return split_direct(*h_, dirs_, faces_, frac_);
    case PutHost: return {{"pcie", "host", shared}, {"hbm", "kernel", shared}};
    case Unpack: return {{"hbm", "kernel", bytes()}, {"pcie", "sdma", shared}};
    default: return {};
    }
  }
  void launch(void *s, Executor &) const override {
    switch (st_) {
    case PutDirect: h_->split_put_direct(dirs_, frac_, s); break;
    case PutHost: h_->hs_put_host(faces_, frac_, s); break;
    case Wait: h_->hs_wait(dirs_, faces_, s); break;
    case Unpack: h_->hs_unpack(dirs_, faces_, frac_, s); break;
    }
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  Stage st_;
  std::vector<int> dirs_, faces_;
  double frac_;
};

/// host-staged transport: the packed send buffers of every remote direction travel device ->
/// host -> control plane -> host -> device (HaloExchange::host_exchange). A host op: the
/// synchronizer makes the pack complete before it and orders the unpack after it.
class HaloHostXfer : public CpuOp {
public:
  HaloHostXfer(std::shared_ptr<const HaloExchange> h, std::vector<int> dirs)
      : h_(std::move(h)), dirs_(std::move(dirs)) {}
  std::string name() const override { return "he_hostxfer"; }
  std::string kind() const override { return "HaloHostExchange"; }
  double bytes() const override {
    double b = 0;
    for (int i : dirs_) b += 8.0 * double(h_->box_elems(i));
    return b;
  }
  // PCIe copies both ways plus loopback TCP through the hub: ~1 GB/s end to end
  double cost_us() const override { return 50.0 + bytes() / 1.0e3; }
  std::string order_domain() const override { return "host"; }
  void run(Executor &ex) const override {
    // a hardware-free search (e.g. the bench's model seeds, on rank 0 alone) must not enter
    // the collective exchange
    if (ex.simulated()) return ex.host_busy(cost_us());
    h_->host_exchange(dirs_);
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  std::vector<int> dirs_;
};

} // namespace

void HaloExchange::add_relay_part(Graph &g, const std::vector<int> &remote, double frac) {
  // the corner put feeds the corner peer's forward, so my forward is issued after my corner
  // put (never ahead of it on a stream, which could deadlock every rank's symmetric
  // schedule); the direct put runs beside both; the wait needs the direct shares and what my
  // forwarders relayed, then the unpack hands out the credits
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  auto mk = [&](HaloRelay::Stage st) { return std::make_shared<HaloRelay>(self, st, remote, frac); };
  auto putd = mk(HaloRelay::PutDirect), putc = mk(HaloRelay::PutCorner), w = mk(HaloRelay::Wait),
       u = mk(HaloRelay::Unpack);
  // the forward copies by kernel or on the copy engines (CUs left to the direct put; only while
  // the SDMA put variant passed its preflight)
  OpPtr fwd = mk(HaloRelay::Forward);
  if (copyOk_[1])
    fwd = std::make_shared<StaticChoiceOp>(
        "he_rl" + std::to_string(int(std::lround(frac * 100))) + "_forward",
        std::vector<OpPtr>{fwd, mk(HaloRelay::ForwardCopy)});
  g.start_then(putd);
  g.start_then(putc);
  g.then(putc, fwd);
  g.then(putd, w);
  g.then(fwd, w);
  g.then(w, u);
  g.then_finish(u);
}

void HaloExchange::add_hostsplit_part(Graph &g, const std::vector<int> &remote, double frac) {
  // both puts need nothing of this iteration (only the previous iteration's credits); the wait
  // needs both, then the unpack returns both kinds of credit
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  auto mk = [&](HaloHostSplit::Stage st) { return std::make_shared<HaloHostSplit>(self, st, remote, frac); };
  auto putd = mk(HaloHostSplit::PutDirect), puth = mk(HaloHostSplit::PutHost),
       w = mk(HaloHostSplit::Wait), u = mk(HaloHostSplit::Unpack);
  g.start_then(putd);
  g.start_then(puth);
  g.then(putd, w);
  g.then(puth, w);
  g.then(w, u);
  g.then_finish(u);
}

void HaloExchange::add_mixed_part(Graph &g, const std::vector<int> &remote) {
  // A link that one engine cannot fill may carry more with two: when both faces of an axis go
  // to the same peer (a dimension of 2 ranks), the + face goes by CU stores and the - face by
  // the copy engines, concurrently if the search puts the two ops on different streams. Both
  // engines signal the same arrival counters, so one wait and one unpack serve both.
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  std::vector<int> byKernel, byCopy;
  for (int i : remote) {
    const Dir &d = dirs_[i];
    const bool face = (d.dx != 0) + (d.dy != 0) + (d.dz != 0) == 1;
    (face && d.dx + d.dy + d.dz < 0 ? byCopy : byKernel).push_back(i);
  }
  auto w = std::make_shared<HaloWait>(self, remote, "mx");
  auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::UnpackRelease, remote, "mx");
  for (auto &[dirs, st] : {std::pair{byKernel, HaloStageGroup::Put}, std::pair{byCopy, HaloStageGroup::CopyPut}}) {
    if (dirs.empty()) continue;
    auto p = std::make_shared<HaloStageGroup>(self, st, dirs, "mx");
    g.start_then(p);
    g.then(p, w);
  }
  g.then(w, u);
  g.then_finish(u);
}

void HaloExchange::add_chains(Graph &g, const std::vector<int> &dirs, int via) {
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  for (int i : dirs) {
    if (direct_[i] || via != kViaPipe) {
      OpPtr d;
      if (direct_[i]) d = std::make_shared<HaloDirect>(self, i);
      else if (via == kViaPut) d = std::make_shared<HaloPut>(self, i);
      else if (via == kViaPutWide) d = std::make_shared<HaloPut>(self, i, a_.wide_put_blocks);
      else d = std::make_shared<HaloStageGroup>(
               self, via == kViaCopy ? HaloStageGroup::CopyPut : HaloStageGroup::MemcpyPut,
               std::vector<int>{i}, dirs_[i].name());
      g.start_then(d);
      g.then_finish(d);
      continue;
    }
    auto p = std::make_shared<HaloPack>(self, i);
    auto s = std::make_shared<HaloShift>(self, i);
    auto u = std::make_shared<HaloUnpack>(self, opp_[i]);
    g.start_then(p);
    g.then(p, s);
    g.then(s, u);
    g.then_finish(u);
  }
}

void HaloExchange::add_fused(Graph &g, const std::vector<int> &dirs, const std::string &tag,
                             int via) {
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  std::vector<int> local, remote;
  for (int i : dirs) (direct_[i] ? local : remote).push_back(i);
  if (!local.empty()) {
    auto d = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Direct, local,
                                              remote.empty() ? tag : tag + "_self");
    g.start_then(d);
    g.then_finish(d);
  }
  if (remote.empty()) return;
  if (via != kViaPipe) {
    const HaloStageGroup::Stage st =
        via == kViaPut ? HaloStageGroup::Put
        : via == kViaPutWide ? HaloStageGroup::WidePut
        : (via == kViaCopy ? HaloStageGroup::CopyPut : HaloStageGroup::MemcpyPut);
    auto d = std::make_shared<HaloStageGroup>(self, st, remote, tag,
                                              via == kViaPutWide ? a_.wide_put_blocks : 0);
    g.start_then(d);
    g.then_finish(d);
    return;
  }
  auto p = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Pack, remote, tag);
  auto s = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Shift, remote, tag);
  auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Unpack, remote, tag);
  g.start_then(p);
  g.then(p, s);
  g.then(s, u);
  g.then_finish(u);
}

void HaloExchange::add_structure(Graph &g, const std::vector<int> &dirs, int via,
                                 const std::string &pre, const std::string &tagPre) {
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  const std::string &f = a_.fuse;
  const bool singleStage = direct_[dirs.front()] || via != kViaPipe;
  auto subset = [&](const std::vector<int> &v) {
    std::vector<int> r;
    for (int i : v)
      if (std::find(dirs.begin(), dirs.end(), i) != dirs.end()) r.push_back(i);
    return r;
  };
  if (f == "none") {
    add_chains(g, dirs, via);
  } else if (f == "all" || (f == "pack" && singleStage)) {
    // (direct moves and puts have no pack stage: "pack" degenerates to one fused op)
    add_fused(g, dirs, tagPre + "all", via);
  } else if (f == "pack") {
    // fused pack / unpack kernels, per-direction transfers
    auto p = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Pack, dirs, tagPre + "all");
    auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Unpack, dirs, tagPre + "all");
    g.start_then(p);
    g.then_finish(u);
    for (int i : dirs) {
      auto s = std::make_shared<HaloShift>(self, i);
      g.then(p, s);
      g.then(s, u);
    }
  } else if (f == "groups" || f == "choice") {
    // faces and (for 26 neighbours) edges+corners form independent groups; each group is
    // either one chain per direction or one fused chain. With "choice" the search decides
    // (ChoiceOp of two CompoundOps; the group touches no other op, so choosing at the group
    // boundary loses no dependency precision).
    std::vector<std::pair<std::string, std::vector<int>>> groups;
    for (auto &gr : std::vector<std::pair<std::string, std::vector<int>>>{
             {"faces", subset(group_dirs(1))}, {"small", subset(group_dirs(0))}})
      if (!gr.second.empty()) groups.push_back(gr);
    if (f == "groups") {
      for (auto &gr : groups) add_fused(g, gr.second, tagPre + gr.first, via);
      return;
    }
    // per group: split chains vs one fused chain
    auto grouped = std::make_shared<Graph>();
    for (auto &gr : groups) {
      auto split = std::make_shared<Graph>();
      add_chains(*split, gr.second, via);
      auto fused = std::make_shared<Graph>();
      add_fused(*fused, gr.second, tagPre + gr.first, via);
      std::vector<OpPtr> alts = {
          std::make_shared<StaticCompoundOp>(pre + "he_" + gr.first + "_split", split),
          std::make_shared<StaticCompoundOp>(pre + "he_" + gr.first + "_fused", fused)};
      auto choice = std::make_shared<StaticChoiceOp>(pre + "he_" + gr.first, alts);
      grouped->start_then(choice);
      grouped->then_finish(choice);
    }
    if (groups.size() == 1) {
      auto c = std::make_shared<StaticCompoundOp>(pre + "he_grouped", grouped);
      g.start_then(c);
      g.then_finish(c);
      return;
    }
    // two groups: additionally one chain for every direction (a single launch per stage
    // avoids the two groups' kernels competing for CUs)
    auto all = std::make_shared<Graph>();
    add_fused(*all, dirs, tagPre + "all", via);
    std::vector<OpPtr> top = {std::make_shared<StaticCompoundOp>(pre + "he_grouped", grouped),
                              std::make_shared<StaticCompoundOp>(pre + "he_allfused", all)};
    // remote directions to several peers: one chain per peer as well. Each peer is one xGMI
    // link, so per-peer transfers on different streams use the links in parallel (copy-engine
    // copies and RCCL groups issued on one stream would take them one at a time)
    // Every rank must build the same graph (schedules are broadcast by op name): the split of
    // directions by peer is the same on every rank of a periodic Cartesian grid, so groups are
    // kept in order of their first direction and named after it, never after a rank id.
    std::map<int, std::vector<int>> byPeer;
    for (int i : dirs)
      if (!direct_[i]) byPeer[nbr_[i]].push_back(i);
    if (byPeer.size() > 1 && byPeer.size() < dirs.size()) {
      std::vector<std::vector<int>> groupsByPeer;
      for (const auto &kv : byPeer) groupsByPeer.push_back(kv.second);
      std::sort(groupsByPeer.begin(), groupsByPeer.end());
      auto peers = std::make_shared<Graph>();
      for (const auto &grp : groupsByPeer)
        add_fused(*peers, grp, tagPre + "p" + dirs_[grp.front()].name(), via);
      top.push_back(std::make_shared<StaticCompoundOp>(pre + "he_bypeer", peers));
    }
    auto choice = std::make_shared<StaticChoiceOp>(pre + "he_exchange", top);
    g.start_then(choice);
    g.then_finish(choice);
  } else {
    TZ_THROW("fuse must be none, pack, all, groups or choice (got " << f << ")");
  }
}

void HaloExchange::add_ipc_part(Graph &g, const std::vector<int> &remote, int via) {
  // puts wait only for the credit of the previous iteration, so each rank's puts all complete;
  // the arrival wait runs after them (one spinning kernel per rank, never ahead of its own
  // puts). The copy-engine and wide variants' op names carry "cp_" / "mc_" / "w_" (unique in the
  // expanded graph).
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  const std::string v = via == kViaCopy ? "cp_" : via == kViaMemcpy ? "mc_" : via == kViaPutWide ? "w_" : "";
  auto puts = std::make_shared<Graph>();
  add_structure(*puts, remote, via, v.empty() ? "ipc_" : v);
  auto c = std::make_shared<StaticCompoundOp>("he_" + v + "puts", puts);
  auto w = std::make_shared<HaloWait>(self, remote, v + "remote");
  g.start_then(c);
  g.then(c, w);
  if (ipcGrid_) {
    g.then_finish(w);
  } else {
    // "buffers" mode: my receive buffers are complete after the wait; unpack them
    auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::UnpackRelease, remote, v + "remote");
    g.then(w, u);
    g.then_finish(u);
  }
}

void HaloExchange::add_to_graph(Graph &g) {
  if (!a_.stencil) {
    add_exchange(g);
    return;
  }
  // the exchange as one compound op, shared by both alternatives
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  auto ex = std::make_shared<Graph>();
  add_exchange(*ex);
  auto xchg = std::make_shared<StaticCompoundOp>("he_xchg", ex);
  // split: interior (needs no ghost) runs beside the exchange, the shell after it
  auto split = std::make_shared<Graph>();
  auto interior = std::make_shared<HaloStencil>(self, 0);
  auto shell = std::make_shared<HaloStencil>(self, 1);
  split->start_then(interior);
  split->then_finish(interior);
  split->start_then(xchg);
  split->then(xchg, shell);
  split->then_finish(shell);
  // full: the whole interior after the exchange (one launch)
  auto full = std::make_shared<Graph>();
  auto all = std::make_shared<HaloStencil>(self, 2);
  full->start_then(xchg);
  full->then(xchg, all);
  full->then_finish(all);
  std::vector<OpPtr> alts = {std::make_shared<StaticCompoundOp>("st_split", split),
                             std::make_shared<StaticCompoundOp>("st_after", full)};
  auto c = std::make_shared<StaticChoiceOp>("st_mode", alts);
  g.start_then(c);
  g.then_finish(c);
}

void HaloExchange::add_exchange(Graph &g) {
  // self-neighbour directions are moved directly and remote directions go through RCCL or IPC
  // puts; the local moves form their own op(s), the remote directions get the fuse structure
  // (and the search overlaps the two). With both transports available ("auto" on several
  // ranks) the transport itself is a ChoiceOp the search decides.
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) (direct_[i] ? local : remote).push_back(i);
  if (remote.empty()) {
    add_structure(g, all_dirs(), kViaPipe, "");
    return;
  }
  if (!local.empty()) {
    if (a_.fuse == "none") add_chains(g, local, kViaPipe);
    else add_fused(g, local, "self", kViaPipe);
  }
  // graph-only builds (no setup) assume IPC can be mapped
  const bool ipc = useIpc_ && (ipcReady_ || !ready());
  const bool pipe = useRccl_ || a_.transport == "copy";
  if (useHost_ && !pipe && !ipc) {
    // no device transport: pack, the host-staged transfer, unpack (one op each)
    auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
    auto p = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Pack, remote, "host");
    auto x = std::make_shared<HaloHostXfer>(self, remote);
    auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Unpack, remote, "host");
    g.start_then(p);
    g.then(p, x);
    g.then(x, u);
    g.then_finish(u);
    return;
  }
  TZ_CHECK(ipc || pipe, "no transport available for the remote directions");
  // directions that cross nodes: RCCL only, a structure of their own (names prefixed "far_");
  // the IPC alternatives below cover the rest
  if (pipe && ipc) {
    std::vector<int> near, far;
    for (int i : remote) (offNode_.empty() || !offNode_[size_t(i)] ? near : far).push_back(i);
    if (!far.empty()) {
      add_structure(g, far, kViaPipe, "far_", "far_");
      if (near.empty()) return;
      remote = near;
    }
  }
  // the copy-engine variant needs receive buffers ("buffers" mode)
  const bool copy = ipc && useCopy_ && !ipcGrid_;
  std::vector<OpPtr> alts;
  if (pipe) {
    auto gr = std::make_shared<Graph>();
    add_structure(*gr, remote, kViaPipe, "");
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_rccl", gr));
  }
  if (ipc) {
    auto gr = std::make_shared<Graph>();
    add_ipc_part(*gr, remote, kViaPut);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_ipc", gr));
  }
  if (ipc && uses_wide_puts()) {
    auto gr = std::make_shared<Graph>();
    add_ipc_part(*gr, remote, kViaPutWide);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_ipcw", gr));
  }
  // (each copy-engine variant only if it passed its preflight; mixed puts use the SDMA one)
  if (copy && copyOk_[1]) {
    auto gr = std::make_shared<Graph>();
    add_ipc_part(*gr, remote, kViaCopy);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_sdma", gr));
  }
  if (copy && copyOk_[0]) {
    auto mc = std::make_shared<Graph>();
    add_ipc_part(*mc, remote, kViaMemcpy);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_memcpy", mc));
  }
  if (copy && copyOk_[1]) {
    auto mx = std::make_shared<Graph>();
    add_mixed_part(*mx, remote);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_mixed", mx));
  }
  if (uses_hostsplit()) {
    if (a_.hostsplit == "force") alts.clear();
    for (double f : a_.hostsplit_fracs) {
      auto gr = std::make_shared<Graph>();
      add_hostsplit_part(*gr, remote, f);
      alts.push_back(std::make_shared<StaticCompoundOp>(
          "he_via_hs" + std::to_string(int(std::lround(f * 100))), gr));
    }
  }
  if (uses_relay() && a_.hostsplit != "force") {
    if (a_.relay == "force") alts.clear();
    for (double f : a_.relay_fracs) {
      auto gr = std::make_shared<Graph>();
      add_relay_part(*gr, remote, f);
      alts.push_back(std::make_shared<StaticCompoundOp>(
          "he_via_relay" + std::to_string(int(std::lround(f * 100))), gr));
    }
  }
  if (alts.size() > 1) {
    auto c = std::make_shared<StaticChoiceOp>("he_remote", alts);
    g.start_then(c);
    g.then_finish(c);
  } else if (a_.relay == "force" || a_.hostsplit == "force") {
    g.start_then(alts.front());
    g.then_finish(alts.front());
  } else if (ipc) {
    add_ipc_part(g, remote, kViaPut);
  } else {
    add_structure(g, remote, kViaPipe, "");
  }
}

} // namespace tz
