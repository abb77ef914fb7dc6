#include "workloads.hpp"

#include "core/numeric.hpp"
#include "core/util.hpp"
#include "hip/hip_runtime.hpp"
#include "hip/rccl_comm.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <map>
#include <cstdlib>
#include <cstring>

namespace tz {

Json HaloArgs::json() const {
  Json j;
  j["nx"] = nx;
  j["ny"] = ny;
  j["nz"] = nz;
  j["nq"] = nq;
  j["ghost"] = ghost;
  j["neighbors"] = neighbors;
  j["order"] = order;
  j["transport"] = transport;
  j["fuse"] = fuse;
  j["comms"] = comms;
  j["rank"] = rank;
  j["size"] = size;
  j["px"] = px;
  j["py"] = py;
  j["pz"] = pz;
  j["pitch_pad"] = pitch_pad;
  j["ghost_align"] = ghost_align;
  j["stencil"] = stencil;
  return j;
}

std::string HaloExchange::Dir::name() const {
  return "dx" + std::to_string(dx) + "_dy" + std::to_string(dy) + "_dz" + std::to_string(dz);
}

namespace {

// byte-cost model for the simulator: ~5 TB/s effective HBM stream + launch latency
double copy_cost_us(double bytes) { return 3.0 + bytes / 5.0e6; }

class HaloPack : public GpuOp {
public:
  HaloPack(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_pack_" + h_->dir(i_).name(); }
  std::string kind() const override { return "HaloPack"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  double cost_us() const override { return copy_cost_us(bytes()); }
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
  void launch(void *s, Executor &) const override { h_->direct(i_, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
};

/// ipc transport: pack-free put of one direction into the neighbour's grid + arrival signal
class HaloPut : public GpuOp {
public:
  HaloPut(std::shared_ptr<const HaloExchange> h, int i) : h_(std::move(h)), i_(i) {}
  std::string name() const override { return "he_put_" + h_->dir(i_).name(); }
  std::string kind() const override { return "HaloPut"; }
  double bytes() const override { return 2.0 * 8.0 * double(h_->box_elems(i_)); }
  // peer stores over one xGMI link (~60 GB/s effective)
  double cost_us() const override { return 4.0 + bytes() / 2.0 / 6.0e4; }
  void launch(void *s, Executor &) const override { h_->put_group({i_}, s); }

private:
  std::shared_ptr<const HaloExchange> h_;
  int i_;
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
  enum Stage { Pack, Shift, Unpack, Direct, Put, UnpackRelease, CopyPut };
  HaloStageGroup(std::shared_ptr<const HaloExchange> h, Stage st, std::vector<int> dirs, std::string tag)
      : h_(std::move(h)), st_(st), dirs_(std::move(dirs)), tag_(std::move(tag)) {}
  std::string name() const override {
    static const char *pre[] = {"he_pack_", "he_shift_", "he_unpack_", "he_direct_", "he_put_",
                                "he_unpack_", "he_copyput_"};
    return pre[st_] + tag_;
  }
  std::string kind() const override {
    static const char *k[] = {"HaloPackGroup", "HaloShiftGroup", "HaloUnpackGroup",
                              "HaloDirectGroup", "HaloPutGroup", "HaloUnpackGroup",
                              "HaloCopyPutGroup"};
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
  void launch(void *s, Executor &ex) const override {
    if (st_ == Pack) h_->pack_group(dirs_, s);
    else if (st_ == Shift) h_->shift_group(dirs_, s, ex.stream_index(s));
    else if (st_ == Unpack) h_->unpack_group(dirs_, s);
    else if (st_ == Direct) h_->direct_group(dirs_, s);
    else if (st_ == Put) h_->put_group(dirs_, s);
    else if (st_ == CopyPut) h_->copy_put_group(dirs_, s);
    else h_->ipc_unpack_group(dirs_, s);
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  Stage st_;
  std::vector<int> dirs_;
  std::string tag_;
};

} // namespace

HaloExchange::HaloExchange(HaloArgs a) : a_(std::move(a)) {
  TZ_CHECK(a_.nx > 0 && a_.ny > 0 && a_.nz > 0 && a_.nq > 0 && a_.ghost > 0, "bad halo extents");
  TZ_CHECK(a_.ghost <= a_.nx && a_.ghost <= a_.ny && a_.ghost <= a_.nz, "ghost wider than domain");
  TZ_CHECK(a_.neighbors == 6 || a_.neighbors == 26, "neighbors must be 6 or 26");
  TZ_CHECK(a_.order == "xyzq" || a_.order == "qxyz", "order must be xyzq or qxyz");
  TZ_CHECK(a_.rank >= 0 && a_.rank < a_.size, "bad rank");
  TZ_CHECK(a_.pitch_pad >= 0 && a_.pitch_pad % 16 == 0, "pitch_pad must be a multiple of 16");
  TZ_CHECK(a_.ghost_align == 0 || a_.ghost_align == 8 || a_.ghost_align == 16,
           "ghost_align must be 0, 8 or 16");

  // rank grid: prime factors (descending) multiply the currently smallest dimension, ties to
  // the later dimension (reference halo_run_strategy.hpp:80-98: 2 -> 1x1x2, 4 -> 1x2x2)
  if (a_.px <= 0 || a_.py <= 0 || a_.pz <= 0) {
    int d[3] = {1, 1, 1};
    for (int64_t p : prime_factors(a_.size)) {
      int best = 2;
      for (int k = 2; k >= 0; --k)
        if (d[k] < d[best]) best = k;
      d[best] *= int(p);
    }
    a_.px = d[0];
    a_.py = d[1];
    a_.pz = d[2];
  }
  TZ_CHECK(a_.px * a_.py * a_.pz == a_.size, "rank grid does not match size");
  cx_ = a_.rank % a_.px;
  cy_ = (a_.rank / a_.px) % a_.py;
  cz_ = a_.rank / (a_.px * a_.py);

  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int k = (dx != 0) + (dy != 0) + (dz != 0);
        if (k == 0) continue;
        if (a_.neighbors == 6 && k != 1) continue;
        dirs_.push_back({dx, dy, dz});
      }
  for (size_t i = 0; i < dirs_.size(); ++i) {
    for (size_t j = 0; j < dirs_.size(); ++j)
      if (dirs_[j].dx == -dirs_[i].dx && dirs_[j].dy == -dirs_[i].dy && dirs_[j].dz == -dirs_[i].dz)
        opp_.push_back(int(j));
    nbr_.push_back(coord_to_rank(cx_ + dirs_[i].dx, cy_ + dirs_[i].dy, cz_ + dirs_[i].dz));
  }

  const int64_t X = a_.nx + 2 * a_.ghost, Y = a_.ny + 2 * a_.ghost, Z = a_.nz + 2 * a_.ghost;
  if (a_.order == "xyzq") {
    // interior rows (and so the inner ends of the x ghost runs) start on a 64-B sector, or on
    // a ghost_align boundary
    const int64_t al = a_.ghost_align > 8 ? a_.ghost_align : 8;
    xoff_ = (al - a_.ghost % al) % al;
    pitch_ = round_up(xoff_ + X, 16) + a_.pitch_pad; // rows are whole 128-B lines
    sy_ = pitch_;
    sz_ = pitch_ * Y;
    sq_ = sz_ * Z;
    gridElems_ = size_t(sq_ * a_.nq);
  } else {
    // (q,x) runs are contiguous, so an x-face row is ONE nq*ghost run (72 B for 3x3) instead of
    // nq runs 4 KB apart (XYZQ). Rows are padded to whole 128-B lines and the x padding is
    // chosen so that (1) each of the four x runs (interior low/high, ghost low/high) touches as
    // few 128-B lines as possible — every x-face row then costs one line fetch — and (2) the
    // interior run is 16-B aligned (dwordx4 y/z-face rows), preferring 128-B alignment.
    const int64_t q = a_.nq, g = a_.ghost, n = a_.nx;
    auto lines = [&](int64_t x0, int64_t len) { // 128-B lines touched by elements [x0,x0+len)
      const int64_t b0 = x0 * 8, b1 = (x0 + len) * 8 - 1;
      return b1 / 128 - b0 / 128 + 1;
    };
    int64_t best = -1, bestCost = 0;
    for (int64_t off = 0; off < 16; ++off) {
      if ((q * (off + g)) % 2 != 0) continue;
      int64_t cost = lines(q * (off + g), q * g) + lines(q * (off + n), q * g) + lines(q * off, q * g) +
                     lines(q * (off + n + g), q * g);
      cost = cost * 4 + ((q * (off + g)) % 16 == 0 ? 0 : ((q * (off + g)) % 8 == 0 ? 1 : 2));
      if (best < 0 || cost < bestCost) {
        best = off;
        bestCost = cost;
      }
    }
    xoff_ = best < 0 ? 0 : best;
    if (a_.ghost_align > 0) {
      // instead: the smallest padding that puts the inner ends of both x ghost runs on
      // ghost_align boundaries (ghost-low ends, ghost-high starts there when q*n is a multiple
      // of it); direct moves then widen the x ghost writes over the row padding to whole units
      for (int64_t off = 0; off < 2 * a_.ghost_align; ++off)
        if ((q * (off + g)) % a_.ghost_align == 0) {
          xoff_ = off;
          break;
        }
    }
    pitch_ = round_up(int64_t(a_.nq) * (xoff_ + X), 16) + a_.pitch_pad;
    sy_ = pitch_;
    sz_ = pitch_ * Y;
    sq_ = 1;
    gridElems_ = size_t(sz_ * Z);
  }
  const std::string &t = a_.transport;
  TZ_CHECK(t == "auto" || t == "direct" || t == "copy" || t == "rccl" || t == "ipc",
           "unknown transport " << t);
  if (t == "copy" || t == "direct") {
    for (int n : nbr_) TZ_CHECK(n == a_.rank, t << " transport needs self-neighbours (1 rank)");
  }
  // per direction: direct move (self-neighbour under auto/direct/ipc), IPC put (remote under
  // ipc) or pack -> transfer -> unpack
  for (int i = 0; i < ndirs(); ++i) {
    const bool self = nbr_[i] == a_.rank;
    direct_.push_back((t == "direct" || t == "auto" || t == "ipc") && self);
    ipc_.push_back((t == "ipc" || t == "auto") && !self);
    pipe_.push_back(!direct_[i] && (t == "rccl" || t == "copy" || t == "auto"));
  }
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) useDirect_ = true;
    if (ipc_[i]) useIpc_ = true;
    if (pipe_[i] && t != "copy") useRccl_ = true;
  }
  ipcGrid_ = gridElems_ * sizeof(double) < (size_t(2) << 30);
  if (const char *v = std::getenv("TZ_IPC_GRID")) ipcGrid_ = std::atoi(v) != 0;
  // copy-engine puts (buffers mode only): on unless TZ_IPC_COPY=0
  useCopy_ = useIpc_;
  if (const char *v = std::getenv("TZ_IPC_COPY")) useCopy_ = useCopy_ && std::atoi(v) != 0;
}

HaloExchange::~HaloExchange() {
  for (void *p : opened_) hipIpcCloseMemHandle(p);
  if (flags_) hipFree(flags_);
}

int HaloExchange::coord_to_rank(int x, int y, int z) const {
  auto w = [](int v, int n) { return ((v % n) + n) % n; };
  return w(x, a_.px) + a_.px * (w(y, a_.py) + a_.py * w(z, a_.pz));
}

static void axis_range(int d, int n, int g, bool ghost, int &lo, int &ext) {
  if (d == 0) {
    lo = g;
    ext = n;
  } else if (d < 0) {
    lo = ghost ? 0 : g;
    ext = g;
  } else {
    lo = ghost ? n + g : n;
    ext = g;
  }
}

static kern::BoxDesc make_box(const HaloArgs &a, const HaloExchange::Dir &d, bool ghost,
                              int64_t xoff, int64_t sy, int64_t sz, int64_t sq) {
  int x0, ex, y0, ey, z0, ez;
  axis_range(d.dx, a.nx, a.ghost, ghost, x0, ex);
  axis_range(d.dy, a.ny, a.ghost, ghost, y0, ey);
  axis_range(d.dz, a.nz, a.ghost, ghost, z0, ez);
  kern::BoxDesc b;
  if (a.order == "xyzq") {
    b.grid_off = z0 * sz + y0 * sy + x0 + xoff;
    b.len = ex;
    b.n1 = ey;
    b.n2 = ez;
    b.n3 = a.nq;
    b.s1 = sy;
    b.s2 = sz;
    b.s3 = sq;
  } else {
    b.grid_off = int64_t(a.nq) * (x0 + xoff) + y0 * sy + z0 * sz;
    b.len = a.nq * ex;
    b.n1 = ey;
    b.n2 = ez;
    b.n3 = 1;
    b.s1 = sy;
    b.s2 = sz;
    b.s3 = 0;
  }
  return b;
}

kern::BoxDesc HaloExchange::pack_box(int i) const {
  kern::BoxDesc b = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
  if (!send_.empty()) b.buf = send_[i].as<double>();
  return b;
}

kern::BoxDesc HaloExchange::unpack_box(int i) const {
  kern::BoxDesc b = make_box(a_, dirs_[i], true, xoff_, sy_, sz_, sq_);
  if (!recv_.empty()) b.buf = recv_[i].as<double>();
  return b;
}

size_t HaloExchange::box_elems(int i) const {
  kern::BoxDesc b = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
  return size_t(b.len) * b.n1 * b.n2 * b.n3;
}

double HaloExchange::exchange_bytes() const {
  double s = 0;
  for (int i = 0; i < ndirs(); ++i) s += 8.0 * double(box_elems(i));
  return s;
}

kern::HaloGeom HaloExchange::geom() const {
  kern::HaloGeom g;
  g.order = a_.order == "xyzq" ? 0 : 1;
  g.xoff = xoff_;
  g.sy = sy_;
  g.sz = sz_;
  g.sq = sq_;
  g.nx = a_.nx;
  g.ny = a_.ny;
  g.nz = a_.nz;
  g.nq = a_.nq;
  g.g = a_.ghost;
  g.cx = cx_;
  g.cy = cy_;
  g.cz = cz_;
  g.px = a_.px;
  g.py = a_.py;
  g.pz = a_.pz;
  g.neighbors = a_.neighbors;
  return g;
}

void HaloExchange::setup(Ctrl *ctrl) {
  if (ready()) return;
  if (a_.device >= 0) TZ_HIP(hipSetDevice(a_.device));
  grid_ = DeviceBuffer(gridElems_ * sizeof(double));
  // staging buffers only for pipelined directions (locality is symmetric: direct_[i] ==
  // direct_[opp(i)], so a pipelined shift(i) never touches a direct direction's buffers)
  send_.resize(ndirs());
  recv_.resize(ndirs());
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) continue;
    if (pipe_[i] || (ipc_[i] && useCopy_ && !ipcGrid_)) send_[i] = DeviceBuffer(box_elems(i) * sizeof(double));
    // ipc "buffers" mode needs the receive buffer too (the peer packs straight into it)
    if (pipe_[i] || (ipc_[i] && !ipcGrid_))
      recv_[i] = DeviceBuffer(box_elems(opp_[i]) * sizeof(double));
  }
  if (useIpc_) {
    // collective agreement: if any rank cannot map its peers, nobody uses IPC puts (with a
    // forced "ipc" transport that is an error; with "auto" RCCL remains)
    const std::string why = setup_ipc(ctrl);
    // agreement (and the barrier before anyone puts: every rank mapped its peers)
    double failed = why.empty() ? 0.0 : 1.0;
    ctrl->allreduce_max(&failed, 1);
    ipcReady_ = failed == 0.0;
    if (!ipcReady_) {
      TZ_LOG(Warn, "ipc transport unavailable" << (why.empty() ? " on another rank" : ": " + why));
      TZ_CHECK(a_.transport != "ipc", "ipc transport requested but unavailable: " << why);
    }
  }
  count_ = DeviceBuffer(sizeof(unsigned long long));
  if (a_.stencil) {
    out_ = DeviceBuffer(gridElems_ * sizeof(double));
    TZ_HIP(hipMemset(out_.get(), 0, out_.bytes()));
  }
  if (useRccl_) {
    TZ_CHECK(ctrl && ctrl->size() == a_.size, "RCCL transport needs a control plane of size "
                                                  << a_.size);
    const int n = a_.comms > 0 ? a_.comms : kDefaultComms;
    int dev = 0;
    TZ_HIP(hipGetDevice(&dev));
    // collective agreement like IPC: if any rank cannot create its communicators (e.g. several
    // ranks on one GPU: RCCL refuses duplicate devices), nobody uses RCCL. With "auto" the IPC
    // puts remain; a forced "rccl" transport is an error.
    std::string why;
    try {
      comms_ = make_rccl_comms(*ctrl, dev, n);
    } catch (const std::exception &e) {
      why = e.what();
      comms_.clear();
    }
    double failed = why.empty() ? 0.0 : 1.0;
    ctrl->allreduce_max(&failed, 1);
    if (failed != 0.0) {
      comms_.clear();
      TZ_LOG(Warn, "RCCL transport unavailable" << (why.empty() ? " on another rank" : ": " + why));
      TZ_CHECK(a_.transport == "auto" && useIpc_ && ipcReady_,
               "RCCL transport unavailable and no IPC fallback: " << why);
      useRccl_ = false;
      for (int i = 0; i < ndirs(); ++i) {
        if (pipe_[i]) {
          pipe_[i] = false;
          // (copy-engine puts pack into send_; buffers-mode puts land in recv_)
          if (!(ipc_[i] && useCopy_ && !ipcGrid_)) send_[i] = DeviceBuffer();
          if (ipcGrid_) recv_[i] = DeviceBuffer();
        }
      }
    }
  }
  init_grid();
  if (useIpc_ && ipcReady_) {
    // a peer's preflight puts land in my ghosts: my init_grid must be complete before anyone
    // puts, and theirs before my check (otherwise their init overwrites what I delivered)
    TZ_HIP(hipDeviceSynchronize());
    ctrl->barrier();
    ipc_preflight(ctrl);
  }
  TZ_HIP(hipDeviceSynchronize());
  if (useIpc_ && ipcReady_) ctrl->barrier();
}

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

void HaloExchange::init_grid(void *stream) {
  TZ_CHECK(ready(), "halo not set up");
  kern::halo_init(grid(), geom(), stream);
  // synchronous: schedules run on non-blocking streams that do not order after `stream`
  TZ_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

uint64_t HaloExchange::check_grid(void *stream) {
  TZ_CHECK(ready(), "halo not set up");
  hipStream_t s = static_cast<hipStream_t>(stream);
  TZ_HIP(hipMemsetAsync(count_.get(), 0, sizeof(unsigned long long), s));
  kern::halo_check(grid(), geom(), count_.as<unsigned long long>(), stream);
  unsigned long long n = 0;
  TZ_HIP(hipMemcpyAsync(&n, count_.get(), sizeof(n), hipMemcpyDeviceToHost, s));
  TZ_HIP(hipStreamSynchronize(s));
  return n;
}

void HaloExchange::check_pipelined(int i) const {
  TZ_CHECK(i >= 0 && i < ndirs(), "direction " << i << " out of range");
  TZ_CHECK(!direct_[i], "direction " << dirs_[i].name()
                                     << " uses the direct transport (no pack/transfer/unpack)");
  TZ_CHECK(pipe_[i] || ipc_[i], "direction " << dirs_[i].name() << " has no staging buffers");
  TZ_CHECK(ready(), "halo not set up");
}

void HaloExchange::pack(int i, void *stream) const {
  check_pipelined(i);
  kern::box_copy(grid(), pack_box(i), false, stream);
}

void HaloExchange::unpack(int i, void *stream) const {
  check_pipelined(i);
  kern::box_copy(grid(), unpack_box(i), true, stream);
}

const RcclComm &HaloExchange::comm_for(int streamIdx, int dir) const {
  TZ_CHECK(!comms_.empty(), "no RCCL communicators");
  // every rank runs the same schedule, so an op lands on the same logical stream, hence the
  // same communicator, on every rank, and each communicator sees its operations in the same
  // order everywhere (RCCL's matching rule)
  const int k = streamIdx >= 0 ? streamIdx : dir;
  return *comms_[size_t(k) % comms_.size()];
}

void HaloExchange::shift(int i, void *stream, int streamIdx) const {
  check_pipelined(i);
  // send my slab facing d to nbr(d); receive nbr(-d)'s slab facing d into my ghost on side -d
  const int o = opp_[i];
  const size_t n = box_elems(i);
  if (useRccl_) {
    const RcclComm &c = comm_for(streamIdx, i);
    c.sendrecv(send_[i].get(), n, nbr_[i], recv_[o].get(), n, nbr_[o], 1, stream);
  } else {
    // self neighbour: device copy kernel (captures as a kernel node, unlike hipMemcpyAsync)
    kern::CopyDesc c{recv_[o].get(), send_[i].get(), n * sizeof(double)};
    kern::copy_many(&c, 1, stream);
  }
}

std::vector<int> HaloExchange::all_dirs() const {
  std::vector<int> v;
  for (int i = 0; i < ndirs(); ++i) v.push_back(i);
  return v;
}

std::vector<int> HaloExchange::group_dirs(int k) const {
  // k = 1: faces, k = 2: edges, k = 3: corners, k = 0: edges + corners
  std::vector<int> v;
  for (int i = 0; i < ndirs(); ++i) {
    const int a = (dirs_[i].dx != 0) + (dirs_[i].dy != 0) + (dirs_[i].dz != 0);
    if (a == k || (k == 0 && a >= 2)) v.push_back(i);
  }
  return v;
}

void HaloExchange::pack_group(const std::vector<int> &dirs, void *stream) const {
  std::vector<kern::BoxDesc> bs;
  for (int i : dirs) {
    check_pipelined(i);
    bs.push_back(pack_box(i));
  }
  for (size_t k = 0; k < bs.size(); k += kern::kMaxBoxes)
    kern::box_copy_many(grid(), bs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, bs.size() - k)),
                        false, stream);
}

void HaloExchange::unpack_group(const std::vector<int> &dirs, void *stream) const {
  // the ghosts filled by the shifts of `dirs` are those on the opposite sides
  std::vector<kern::BoxDesc> bs;
  for (int i : dirs) {
    check_pipelined(i);
    bs.push_back(unpack_box(opp_[i]));
  }
  for (size_t k = 0; k < bs.size(); k += kern::kMaxBoxes)
    kern::box_copy_many(grid(), bs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, bs.size() - k)),
                        true, stream);
}

void HaloExchange::shift_group(const std::vector<int> &dirs, void *stream, int streamIdx) const {
  if (dirs.empty()) return;
  for (int i : dirs) check_pipelined(i);
  if (useRccl_) {
    std::vector<RcclComm::Xfer> xs;
    for (int i : dirs) {
      const int o = opp_[i];
      const size_t n = box_elems(i);
      xs.push_back({send_[i].get(), n, nbr_[i], recv_[o].get(), n, nbr_[o]});
    }
    comm_for(streamIdx, dirs.front()).exchange(xs, 1, stream);
  } else {
    std::vector<kern::CopyDesc> cs;
    for (int i : dirs) cs.push_back({recv_[opp_[i]].get(), send_[i].get(), box_elems(i) * sizeof(double)});
    for (size_t k = 0; k < cs.size(); k += kern::kMaxBoxes)
      kern::copy_many(cs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, cs.size() - k)), stream);
  }
}

void HaloExchange::direct_group(const std::vector<int> &dirs, void *stream) const {
  std::vector<kern::MoveDesc> ms;
  for (int i : dirs) {
    TZ_CHECK(i >= 0 && i < ndirs() && direct_[i], "direction " << i << " is not a direct (self) transfer");
    TZ_CHECK(ready(), "halo not set up");
    // my slab facing d lands in nbr(d)'s ghost on side -d (self-neighbours: my own grid)
    const kern::BoxDesc s = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
    const kern::BoxDesc d = make_box(a_, dirs_[opp_[i]], true, xoff_, sy_, sz_, sq_);
    kern::MoveDesc m;
    m.src = grid();
    m.dst = grid();
    m.src_off = s.grid_off;
    m.dst_off = d.grid_off;
    m.s1 = s.s1;
    m.s2 = s.s2;
    m.s3 = s.s3;
    m.len = s.len;
    m.n1 = s.n1;
    m.n2 = s.n2;
    m.n3 = s.n3;
    if (a_.ghost_align > 0) widen_to_sectors(dirs_[opp_[i]].dx, m);
    ms.push_back(m);
  }
  for (size_t k = 0; k < ms.size(); k += kern::kMaxBoxes)
    kern::box_move_many(ms.data() + k, int(std::min<size_t>(kern::kMaxBoxes, ms.size() - k)), stream);
}

void HaloExchange::widen_to_sectors(int ghostDx, kern::MoveDesc &m) const {
  // A move whose destination is an x ghost run (side -x: ghost-low, +x: ghost-high) writes a
  // few elements less than whole 64-B sectors; the rest of those sectors is row padding (x < 0
  // or x >= n + 2g), whose contents nobody reads. Widening source and destination rows over
  // that padding turns every x-face write into full-sector writes (a partially written sector
  // costs the memory a read-modify-write). Row strides are multiples of 16 elements, so the
  // alignment of the first row holds for every row.
  if (ghostDx == 0) return;
  const int64_t rowLen = pitch_; // elements per (y[,q]) row, a multiple of 16
  if (ghostDx < 0) {
    const int64_t A = a_.ghost_align;
    const int64_t x0 = m.dst_off % rowLen; // ghost-low: padding [0, x0) before it
    const int64_t e = m.dst_off % A;
    if (e > x0) return;
    m.src_off -= e;
    m.dst_off -= e;
    m.len += int32_t(e);
  } else {
    const int64_t A = a_.ghost_align;
    const int64_t end = m.dst_off % rowLen + m.len; // ghost-high: padding [end, rowLen) after
    const int64_t e = (A - (m.dst_off + m.len) % A) % A;
    if (end + e > rowLen) return;
    m.len += int32_t(e);
  }
}

std::vector<int> HaloExchange::pipelined_dirs() const {
  std::vector<int> v;
  for (int i = 0; i < ndirs(); ++i)
    if (!direct_[i]) v.push_back(i);
  return v;
}

void HaloExchange::pack_all(void *stream) const { pack_group(pipelined_dirs(), stream); }
void HaloExchange::unpack_all(void *stream) const { unpack_group(pipelined_dirs(), stream); }
void HaloExchange::shift_all(void *stream) const { shift_group(pipelined_dirs(), stream); }

void HaloExchange::add_chains(Graph &g, const std::vector<int> &dirs, int via) {
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  for (int i : dirs) {
    if (direct_[i] || via != kViaPipe) {
      OpPtr d;
      if (direct_[i]) d = std::make_shared<HaloDirect>(self, i);
      else if (via == kViaPut) d = std::make_shared<HaloPut>(self, i);
      else d = std::make_shared<HaloStageGroup>(self, HaloStageGroup::CopyPut, std::vector<int>{i},
                                                dirs_[i].name());
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
    auto d = std::make_shared<HaloStageGroup>(
        self, via == kViaPut ? HaloStageGroup::Put : HaloStageGroup::CopyPut, remote, tag);
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
                                 const std::string &pre) {
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
    add_fused(g, dirs, "all", via);
  } else if (f == "pack") {
    // fused pack / unpack kernels, per-direction transfers
    auto p = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Pack, dirs, "all");
    auto u = std::make_shared<HaloStageGroup>(self, HaloStageGroup::Unpack, dirs, "all");
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
      for (auto &gr : groups) add_fused(g, gr.second, gr.first, via);
      return;
    }
    // per group: split chains vs one fused chain
    auto grouped = std::make_shared<Graph>();
    for (auto &gr : groups) {
      auto split = std::make_shared<Graph>();
      add_chains(*split, gr.second, via);
      auto fused = std::make_shared<Graph>();
      add_fused(*fused, gr.second, gr.first, via);
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
    add_fused(*all, dirs, "all", via);
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
      for (const auto &grp : groupsByPeer) add_fused(*peers, grp, "p" + dirs_[grp.front()].name(), via);
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
  // puts). The copy-engine variant's op names carry "cp_" (unique in the expanded graph).
  auto self = std::const_pointer_cast<const HaloExchange>(shared_from_this());
  const std::string v = via == kViaCopy ? "cp_" : "";
  auto puts = std::make_shared<Graph>();
  add_structure(*puts, remote, via, via == kViaCopy ? "cp_" : "ipc_");
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

kern::StencilBox HaloExchange::stencil_box(int x0, int x1, int y0, int y1, int z0, int z1) const {
  // cells [x0,x1) x [y0,y1) x [z0,z1) of the interior (interior coordinates)
  kern::StencilBox b;
  b.in = grid();
  b.out = out_.as<double>();
  const int64_t g = a_.ghost;
  if (a_.order == "xyzq") {
    b.base = (z0 + g) * sz_ + (y0 + g) * sy_ + (x0 + g) + xoff_;
    b.row = x1 - x0;
    b.xs = 1;
    b.so = sq_;
    b.nouter = a_.nq;
  } else {
    b.base = int64_t(a_.nq) * (x0 + g + xoff_) + (y0 + g) * sy_ + (z0 + g) * sz_;
    b.row = a_.nq * (x1 - x0);
    b.xs = a_.nq;
    b.so = 0;
    b.nouter = 1;
  }
  b.sy = sy_;
  b.sz = sz_;
  b.ny = y1 - y0;
  b.nz = z1 - z0;
  return b;
}

void HaloExchange::stencil(int region, void *stream) const {
  TZ_CHECK(ready() && out_.get(), "stencil mode not set up");
  const int X = a_.nx, Y = a_.ny, Z = a_.nz;
  std::vector<kern::StencilBox> boxes;
  if (region == 2) {
    boxes.push_back(stencil_box(0, X, 0, Y, 0, Z));
  } else if (region == 0) {
    // full rows with the first / last x cell masked: rows stay 16-B aligned
    if (X > 2 && Y > 2 && Z > 2) {
      kern::StencilBox b = stencil_box(0, X, 1, Y - 1, 1, Z - 1);
      b.m0 = b.m1 = b.xs;
      boxes.push_back(b);
    }
  } else {
    // the shell: two z planes, two y slabs between them, two x slabs inside those
    boxes.push_back(stencil_box(0, X, 0, Y, 0, 1));
    if (Z > 1) boxes.push_back(stencil_box(0, X, 0, Y, Z - 1, Z));
    if (Z > 2) {
      boxes.push_back(stencil_box(0, X, 0, 1, 1, Z - 1));
      if (Y > 1) boxes.push_back(stencil_box(0, X, Y - 1, Y, 1, Z - 1));
      if (Y > 2) {
        boxes.push_back(stencil_box(0, 1, 1, Y - 1, 1, Z - 1));
        if (X > 1) boxes.push_back(stencil_box(X - 1, X, 1, Y - 1, 1, Z - 1));
      }
    }
  }
  // thin boxes (the shell's slabs) share one launch; the rest go one by one
  std::vector<kern::StencilBox> thin;
  for (const auto &b : boxes) {
    if (kern::stencil_thin(b)) thin.push_back(b);
    else kern::stencil7(b, true, stream);
  }
  if (!thin.empty()) kern::stencil7_thin_many(thin.data(), int(thin.size()), stream);
}

uint64_t HaloExchange::check_stencil(void *stream) {
  TZ_CHECK(ready() && out_.get(), "stencil mode not set up");
  hipStream_t s = static_cast<hipStream_t>(stream);
  TZ_HIP(hipMemsetAsync(count_.get(), 0, sizeof(unsigned long long), s));
  kern::stencil_check(out_.as<double>(), geom(), count_.as<unsigned long long>(), stream);
  unsigned long long n = 0;
  TZ_HIP(hipMemcpyAsync(&n, count_.get(), sizeof(n), hipMemcpyDeviceToHost, s));
  TZ_HIP(hipStreamSynchronize(s));
  return n;
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
  TZ_CHECK(ipc || pipe, "no transport available for the remote directions");
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
  if (copy) {
    auto gr = std::make_shared<Graph>();
    add_ipc_part(*gr, remote, kViaCopy);
    alts.push_back(std::make_shared<StaticCompoundOp>("he_via_sdma", gr));
  }
  if (alts.size() > 1) {
    auto c = std::make_shared<StaticChoiceOp>("he_remote", alts);
    g.start_then(c);
    g.then_finish(c);
  } else if (ipc) {
    add_ipc_part(g, remote, kViaPut);
  } else {
    add_structure(g, remote, kViaPipe, "");
  }
}

} // namespace tz
