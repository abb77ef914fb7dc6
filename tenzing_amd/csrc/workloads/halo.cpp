// Halo workload: arguments, rank grid and grid layout, setup, and the pack / unpack / RCCL
// shift / direct-move operations (reference src/halo_exchange/ops_halo_exchange.cu).
// IPC / SDMA transport: halo_ipc.cpp; op graph: halo_graph.cpp; stencil: halo_stencil.cpp.
#include "halo_internal.hpp"

#include <functional>
#include <map>

#include "core/health.hpp"
#include "core/solve.hpp"

#include <algorithm>
#include <chrono>
#include <thread>

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
  j["relay"] = relay;
  Json f = Json::array();
  for (double v : relay_fracs) f.push_back(v);
  j["relay_fracs"] = f;
  j["hostsplit"] = hostsplit;
  Json hf = Json::array();
  for (double v : hostsplit_fracs) hf.push_back(v);
  j["hostsplit_fracs"] = hf;
  j["hostsplit_chunks"] = hostsplit_chunks;
  j["wide_puts"] = wide_puts;
  j["wide_put_blocks"] = wide_put_blocks;
  j["ipc_grid"] = ipc_grid;
  j["copy_puts"] = copy_puts;
  j["copy_engines"] = copy_engines;
  j["move_pairs"] = move_pairs;
  j["grid_memory"] = grid_memory;
  j["node_tag"] = node_tag;
  return j;
}

std::string HaloExchange::Dir::name() const {
  return "dx" + std::to_string(dx) + "_dy" + std::to_string(dy) + "_dz" + std::to_string(dz);
}


HaloExchange::HaloExchange(HaloArgs a) : a_(std::move(a)) {
  TZ_CHECK(a_.nx > 0 && a_.ny > 0 && a_.nz > 0 && a_.nq > 0 && a_.ghost > 0, "bad halo extents");
  // the verification values (halo_value, kernels/halo_kernels.hip) pack (gen, q, z, y, x) into
  // the 53 exact bits of a double: q in 3 bits below the generation, 16 bits per global axis
  TZ_CHECK(a_.nq <= 8, "at most 8 quantities per cell (got " << a_.nq
                                                             << "): the grid checks encode q in 3 bits");
  TZ_CHECK(a_.ghost <= a_.nx && a_.ghost <= a_.ny && a_.ghost <= a_.nz, "ghost wider than domain");
  TZ_CHECK(a_.neighbors == 6 || a_.neighbors == 26, "neighbors must be 6 or 26");
  TZ_CHECK(a_.order == "xyzq" || a_.order == "qxyz", "order must be xyzq or qxyz");
  TZ_CHECK(a_.rank >= 0 && a_.rank < a_.size, "bad rank");
  TZ_CHECK(a_.ghost_align >= -2 && (a_.ghost_align <= 0 || a_.ghost_align == 8 || a_.ghost_align == 16),
           "ghost_align must be -2 (auto), -1 (x = 0 at the row start), 0, 8 or 16");
  // auto: line-aligned ghost runs in both orders. In QXYZ a row's ghost and source runs (9
  // doubles each) cannot share a line, so each on a line of its own is the minimum traffic. In
  // XYZQ the one-GPU self move is 3 % faster with x = 0 at the row start (profiles/r5_roof/: 90
  // vs 93 us), but line-aligned runs are what the remote puts' sector widening, the widened
  // unpack and the stencil's 16-B interior path rely on; the reference layout (-1) is asked for
  // explicitly where it is wanted (bench.py's reference_layout sub-record)
  if (a_.ghost_align == -2) a_.ghost_align = 16;
  // extra row pitch: whole 64-B sectors (even strides keep the 16-B paths); with line-aligned
  // ghosts whole 128-B lines, which the widened x-ghost writes assume of every row stride
  const int padUnit = a_.ghost_align == 16 ? 16 : 8;
  TZ_CHECK(a_.pitch_pad >= 0 && a_.pitch_pad % padUnit == 0,
           "pitch_pad must be a multiple of " << padUnit << " elements here (got " << a_.pitch_pad << ")");
  TZ_CHECK(a_.wide_puts == "auto" || a_.wide_puts == "on" || a_.wide_puts == "off",
           "wide_puts must be auto, on or off");
  TZ_CHECK(a_.wide_put_blocks >= 1 && a_.wide_put_blocks <= 4096,
           "wide_put_blocks must be in [1, 4096]");

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
    // (ghost_align -1: no padding, x = 0 at the start of the pitched row, as the reference
    // driver lays it out: halo_run_strategy.hpp:49, 63-64)
    const int64_t al = a_.ghost_align > 8 ? a_.ghost_align : 8;
    xoff_ = a_.ghost_align < 0 ? 0 : (al - a_.ghost % al) % al;
    pitch_ = round_up(xoff_ + X, 16) + a_.pitch_pad; // whole 128-B lines (+ pitch_pad)
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
    xoff_ = best < 0 || a_.ghost_align < 0 ? 0 : best;
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
  TZ_CHECK(t == "auto" || t == "direct" || t == "copy" || t == "rccl" || t == "ipc" || t == "host",
           "unknown transport " << t);
  if (t == "copy" || t == "direct") {
    for (int n : nbr_) TZ_CHECK(n == a_.rank, t << " transport needs self-neighbours (1 rank)");
  }
  // per direction: direct move (self-neighbour under auto/direct/ipc/host), IPC put (remote
  // under ipc) or pack -> transfer -> unpack (the transfer: RCCL, a device copy, or the host)
  for (int i = 0; i < ndirs(); ++i) {
    const bool self = nbr_[i] == a_.rank;
    direct_.push_back((t == "direct" || t == "auto" || t == "ipc" || t == "host") && self);
    ipc_.push_back((t == "ipc" || t == "auto") && !self);
    pipe_.push_back(!direct_[i] && (t == "rccl" || t == "copy" || t == "auto" || t == "host"));
  }
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) useDirect_ = true;
    if (ipc_[i]) useIpc_ = true;
    if (pipe_[i] && t != "copy" && t != "host") useRccl_ = true;
    if (pipe_[i] && t == "host") useHost_ = true;
  }
  TZ_CHECK(a_.ipc_grid >= -1 && a_.ipc_grid <= 1, "ipc_grid must be -1 (auto), 0 or 1");
  TZ_CHECK(a_.copy_engines >= 1 && a_.copy_engines <= 8, "copy_engines must be in [1, 8]");
  ipcGrid_ = a_.ipc_grid < 0 ? gridElems_ * sizeof(double) < (size_t(2) << 30) : a_.ipc_grid != 0;
  // In grid mode a receiver hands the credit back as soon as the ghosts arrived, so a sender
  // one iteration ahead may overwrite them. That is fine while nothing reads them between
  // exchanges, but the stencil does: it takes buffers mode, where puts land in receive buffers
  // and the credit waits for the unpack into the grid. (A credit deferred to the next
  // exchange's start removes the slack that keeps puts from waiting on the peer's current
  // iteration; with several ranks time-slicing one GPU that stalled waits for seconds.)
  if (a_.stencil) ipcGrid_ = false;
  // copy-engine puts (buffers mode only)
  useCopy_ = useIpc_ && a_.copy_puts;
  copyEngines_ = a_.copy_engines;

  // relay routing through the corner peer: a 2x2x2 grid (the only single-node grid where the
  // corner and edge-diagonal links idle while both faces of an axis share one link), ipc puts
  // into receive buffers for every face
  TZ_CHECK(a_.relay == "auto" || a_.relay == "off" || a_.relay == "force",
           "relay must be auto, off or force (got " << a_.relay << ")");
  TZ_CHECK(!a_.relay_fracs.empty(), "relay_fracs is empty");
  for (double f : a_.relay_fracs) TZ_CHECK(f > 0.0 && f < 0.5, "relay fraction " << f << " not in (0, 0.5)");
  bool facesIpc = true;
  for (int i : group_dirs(1)) facesIpc = facesIpc && ipc_[i];
  relay_ = a_.relay != "off" && a_.px == 2 && a_.py == 2 && a_.pz == 2 && useIpc_ && !ipcGrid_ && facesIpc;
  TZ_CHECK(a_.relay != "force" || relay_,
           "relay routing forced but needs a 2x2x2 rank grid with ipc puts in buffers mode");
  // host split: like relay routing it splits faces and needs receive buffers (with slack for
  // the second share behind the first)
  TZ_CHECK(a_.hostsplit == "auto" || a_.hostsplit == "off" || a_.hostsplit == "force",
           "hostsplit must be auto, off or force (got " << a_.hostsplit << ")");
  TZ_CHECK(!a_.hostsplit_fracs.empty(), "hostsplit_fracs is empty");
  for (double f : a_.hostsplit_fracs)
    TZ_CHECK(f > 0.0 && f < 1.0, "host share " << f << " not in (0, 1)");
  TZ_CHECK(a_.hostsplit_chunks >= 1 && a_.hostsplit_chunks <= 8,
           "hostsplit_chunks must be 1..8 (got " << a_.hostsplit_chunks << ")");
  hsChunks_ = a_.hostsplit_chunks;
  bool anyFace = false;
  for (int i : group_dirs(1)) anyFace = anyFace || ipc_[i];
  hsOffered_ = a_.hostsplit != "off" && useIpc_ && !ipcGrid_ && anyFace;
  TZ_CHECK(a_.hostsplit != "force" || hsOffered_,
           "host split forced but needs remote faces with ipc puts in buffers mode");
  corner_ = coord_to_rank(cx_ + 1, cy_ + 1, cz_ + 1);
  relayOrigin_ = coord_to_rank(cx_ - 1, cy_ - 1, cz_ - 1);
  fwdTo_.assign(dirs_.size(), -1);
  fwdFrom_.assign(dirs_.size(), -1);
  for (size_t i = 0; i < dirs_.size(); ++i) {
    const Dir &d = dirs_[i];
    // I forward what my origin (r - e) relayed for direction d to r - e + d; what travels to me
    // in direction d was sent by me - d and forwarded by me - d + e
    fwdTo_[i] = coord_to_rank(cx_ - 1 + d.dx, cy_ - 1 + d.dy, cz_ - 1 + d.dz);
    fwdFrom_[i] = coord_to_rank(cx_ - d.dx + 1, cy_ - d.dy + 1, cz_ - d.dz + 1);
  }
}

HaloExchange::~HaloExchange() {
  if (recoveryHook_) remove_recovery_hook(recoveryHook_);
  // teardown: nothing useful to do with an error here
  for (auto &kv : engines_) {
    for (void *e : kv.second.events) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
    for (void *s : kv.second.streams) (void)hipStreamDestroy(static_cast<hipStream_t>(s));
  }
  for (void *p : opened_) (void)hipIpcCloseMemHandle(p);
  if (flags_) (void)hipFree(flags_);
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

kern::BoxDesc halo_detail::make_box(const HaloArgs &a, const HaloExchange::Dir &d, bool ghost,
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
  // (no widening: reading the x-face runs as whole 16-B sectors measured no faster, 48.5-50.1
  // vs 48.4 us for the 26-box pack, profiles/r5_unpack/; partial reads cost no read-modify-write)
  return b;
}

kern::BoxDesc HaloExchange::unpack_box(int i) const {
  kern::BoxDesc b = make_box(a_, dirs_[i], true, xoff_, sy_, sz_, sq_);
  if (!recv_.empty()) b.buf = recv_[i].as<double>();
  // x ghost runs: the unpack's writes may cover the row padding beside them (whole sectors)
  ghost_widening(dirs_[i].dx, b.grid_off, b.len, b.lead, b.trail);
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
  g.gen = gen_;
  return g;
}

void HaloExchange::setup(Ctrl *ctrl) {
  if (ready()) return;
  ctrl_ = ctrl;
  if (a_.device >= 0) TZ_HIP(hipSetDevice(a_.device));
  TZ_CHECK(a_.grid_memory >= -1 && a_.grid_memory <= 1, "grid_memory must be -1 (auto), 0 or 1");
  if (useIpc_ && ctrl && ctrl->size() > 1) {
    // IPC needs the neighbour on this node. A direction whose neighbour runs on another node on
    // ANY rank goes over RCCL on every rank (a shift pairs my send in direction d with my
    // receive from the opposite side: both ends must use one transport), the other remote
    // directions keep the IPC transports. One node: nothing changes.
    const std::vector<std::string> ids = ctrl->allgather(node_identity() + a_.node_tag);
    TZ_CHECK(int(ids.size()) == a_.size, "allgather returned " << ids.size() << " entries");
    std::vector<double> off(size_t(ndirs()), 0.0);
    for (int i = 0; i < ndirs(); ++i)
      if (ipc_[i] && ids[size_t(nbr_[i])] != ids[size_t(a_.rank)]) off[size_t(i)] = 1.0;
    ctrl->allreduce_max(off.data(), int(off.size()));
    offNode_.assign(size_t(ndirs()), 0);
    int n = 0;
    for (int i = 0; i < ndirs(); ++i)
      if (off[size_t(i)] != 0.0) {
        offNode_[size_t(i)] = 1;
        ipc_[i] = false;
        ++n;
      }
    if (n > 0) {
      TZ_CHECK(a_.transport == "auto", "transport " << a_.transport << ": " << n
                   << " directions have a neighbour on another node, which IPC cannot reach "
                      "(transport auto sends them over RCCL)");
      useIpc_ = std::any_of(ipc_.begin(), ipc_.end(), [](bool b) { return b; });
      // relay routing and the host split assume every face is an IPC put
      relay_ = false;
      hsOffered_ = false;
      useCopy_ = useIpc_ && a_.copy_puts;
      TZ_LOG(Info, "halo: " << n << " directions cross nodes (RCCL), "
                            << std::count(ipc_.begin(), ipc_.end(), true) << " stay on IPC");
    }
  }
  // IPC grid mode: the neighbours' puts store into this grid's ghost cells, as into receive
  // buffers in buffers mode (DeviceBuffer's peerWritten note)
  gridFine_ = a_.grid_memory < 0 ? useIpc_ && ipcGrid_ : a_.grid_memory != 0;
  grid_ = DeviceBuffer(gridElems_ * sizeof(double), gridFine_);
  // staging buffers only for pipelined directions (locality is symmetric: direct_[i] ==
  // direct_[opp(i)], so a pipelined shift(i) never touches a direct direction's buffers)
  send_.resize(ndirs());
  recv_.resize(ndirs());
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) continue;
    if (pipe_[i] || (ipc_[i] && useCopy_ && !ipcGrid_)) send_[i] = DeviceBuffer(box_elems(i) * sizeof(double));
    // ipc "buffers" mode needs the receive buffer too (the peer packs straight into it); the
    // slack lets a relayed share (or each chunk of a host share) start on a 128-B boundary
    // behind the direct share
    if (pipe_[i] || (ipc_[i] && !ipcGrid_))
      recv_[i] = DeviceBuffer((box_elems(opp_[i]) + 16 * ((relay_ ? 1 : 0) + (hsOffered_ ? hsChunks_ + 1 : 0))) *
                                  sizeof(double),
                              /*peerWritten=*/ipc_[i] && !ipcGrid_);
  }
  if (relay_) {
    // the shares my origin relays through me: its face boxes have my boxes' shapes
    relayBuf_.resize(ndirs());
    for (int i : relay_faces()) {
      size_t most = 0;
      for (double f : a_.relay_fracs) {
        kern::BoxDesc A, B;
        split_box(make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_), f, A, B);
        most = std::max(most, size_t(B.len) * B.n1 * B.n2 * B.n3);
      }
      relayBuf_[i] = DeviceBuffer(most * sizeof(double), /*peerWritten=*/true);
    }
  }
  // TZ_FAIL_TRANSPORTS=ipc,rccl,rccl_hang: simulated setup / preflight failures (tests of the
  // fallback chain: ipc -> rccl -> host)
  const std::string failEnv = std::getenv("TZ_FAIL_TRANSPORTS") ? std::getenv("TZ_FAIL_TRANSPORTS") : "";
  auto simulated = [&](const std::string &what) {
    return ("," + failEnv + ",").find("," + what + ",") != std::string::npos;
  };
  if (useIpc_) {
    // collective agreement: if any rank cannot map its peers, nobody uses IPC puts (with a
    // forced "ipc" transport that is an error; with "auto" RCCL remains)
    std::string why = setup_ipc(ctrl);
    if (why.empty() && simulated("ipc")) why = "simulated failure (TZ_FAIL_TRANSPORTS)";
    // agreement (and the barrier before anyone puts: every rank mapped its peers)
    double failed = why.empty() ? 0.0 : 1.0;
    ctrl->allreduce_max(&failed, 1);
    ipcReady_ = failed == 0.0;
    if (!ipcReady_) {
      ipcWhy_ = why.empty() ? "failed on another rank" : why;
      TZ_LOG(Warn, "ipc transport unavailable: " << ipcWhy_);
      TZ_CHECK(a_.transport != "ipc", "ipc transport requested but unavailable: " << why);
    }
    if (relay_) {
      // relay routing needs more mappings (corner and edge-diagonal peers): agreed separately,
      // so a failure there costs only the relay alternative
      double bad = relayWhy_.empty() ? 0.0 : 1.0;
      ctrl->allreduce_max(&bad, 1);
      relayReady_ = ipcReady_ && bad == 0.0;
      if (ipcReady_ && !relayReady_) {
        TZ_LOG(Warn, "relay routing unavailable"
                         << (relayWhy_.empty() ? " on another rank" : ": " + relayWhy_));
        TZ_CHECK(a_.relay != "force", "relay routing forced but unavailable: " << relayWhy_);
        if (relayWhy_.empty()) relayWhy_ = "failed on another rank";
      }
    }
  }
  if (hsOffered_ && ipcReady_) {
    // shared host memory for the PCIe share: agreed like the relay mappings (a failure costs
    // only the host-split alternative)
    hsWhy_ = setup_hostsplit(ctrl);
    double bad = hsWhy_.empty() ? 0.0 : 1.0;
    ctrl->allreduce_max(&bad, 1);
    hsReady_ = bad == 0.0;
    if (!hsReady_) {
      if (hsWhy_.empty()) hsWhy_ = "failed on another rank";
      TZ_LOG(Warn, "host split unavailable: " << hsWhy_);
      TZ_CHECK(a_.hostsplit != "force", "host split forced but unavailable: " << hsWhy_);
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
    // ranks on one GPU: RCCL refuses duplicate devices), nobody uses RCCL
    std::string why;
    try {
      if (simulated("rccl")) TZ_THROW("simulated failure (TZ_FAIL_TRANSPORTS)");
      comms_ = make_rccl_comms(*ctrl, dev, n);
    } catch (const std::exception &e) {
      why = e.what();
    }
    double failed = why.empty() ? 0.0 : 1.0;
    ctrl->allreduce_max(&failed, 1);
    if (failed != 0.0) drop_rccl(why.empty() ? "communicator creation failed on another rank" : why);
  }
  init_grid();
  if (useRccl_) {
    // a transfer that could hang or deliver wrong data must show up here, bounded, and not
    // mid-search on every rank: one verified exchange per form the search can build
    const std::string why = rccl_preflight(*ctrl);
    if (!why.empty()) {
      drop_rccl("preflight: " + why);
    } else {
      if (!rcclGraphOk_) TZ_LOG(Warn, "RCCL ops run eagerly only: " << rcclGraphWhy_);
      TZ_LOG(Info, "rccl preflight passed (" << comms_.size() << " communicators of "
                                             << rccl_nranks() << " ranks)"
                                             << (rcclGraphOk_ ? ", " + rcclCaptureNote_ : ", eager only"));
    }
    init_grid();
  }
  if (useIpc_ && ipcReady_) {
    // a peer's preflight puts land in my ghosts: my init_grid must be complete before anyone
    // puts, and theirs before my check (otherwise their init overwrites what I delivered)
    TZ_HIP(hipDeviceSynchronize());
    ctrl->barrier();
    ipc_preflight(ctrl);
    if (ipcReady_ && useCopy_ && !ipcGrid_) copy_preflight(ctrl);
    if (ipcReady_) wide_put_preflight(ctrl);
    if (relay_ && ipcReady_) relay_preflight(ctrl);
    if (hsReady_ && ipcReady_) hostsplit_preflight(ctrl);
  }
  // remote directions left without a working device transport: IPC puts take them, or the
  // host-staged transport (the one that works whenever the control plane does)
  bool piped = false;
  for (int i = 0; i < ndirs(); ++i) piped = piped || pipe_[i];
  if (piped && !useRccl_ && a_.transport != "copy" && !useHost_) {
    if (!off_node_dirs().empty() && useIpc_ && ipcReady_) {
      // off-node directions have no IPC path: the host-staged transport carries every remote
      // direction (one mechanism, agreed by every rank through RCCL's failure agreement)
      ipcReady_ = false;
      ipcWhy_ = "RCCL unavailable for the directions that cross nodes: host-staged transport";
    }
    if (useIpc_ && ipcReady_) {
      for (int i = 0; i < ndirs(); ++i) {
        if (pipe_[i]) {
          pipe_[i] = false;
          // (copy-engine puts pack into send_; buffers-mode puts land in recv_)
          if (!(ipc_[i] && useCopy_ && !ipcGrid_)) send_[i] = DeviceBuffer();
          if (ipcGrid_) recv_[i] = DeviceBuffer();
        }
      }
    } else {
      TZ_CHECK(a_.transport == "auto", "RCCL transport unavailable and no fallback: " << rcclWhy_);
      useHost_ = true;
      TZ_LOG(Warn, "no device transport works (rccl: " << rcclWhy_ << "; ipc: "
                                                     << (useIpc_ ? ipcWhy_ : "not offered")
                                                     << "): the host-staged transport carries "
                                                        "the remote directions");
    }
  }
  TZ_HIP(hipDeviceSynchronize());
  if (useIpc_ && ipcReady_) {
    ctrl->barrier();
    // an aborted run leaves the put / wait counters out of step on some ranks: every rank
    // resets them together before the next candidate (health.hpp)
    recoveryHook_ = add_recovery_hook([this](Ctrl &c) { reset_ipc_counters(&c); });
  }
}

void HaloExchange::drop_rccl(const std::string &why) {
  // abort rather than destroy: a destroy waits for outstanding operations, which after a
  // failed exchange may never complete
  for (auto &c : comms_)
    if (c && !c->aborted()) c->abort();
  comms_.clear();
  useRccl_ = false;
  rcclWhy_ = why;
  TZ_LOG(Warn, "RCCL transport unavailable: " << why);
}

int HaloExchange::rccl_nranks() const { return comms_.empty() ? 0 : comms_.front()->size(); }

std::map<std::string, std::string> HaloExchange::transport_report() const {
  std::map<std::string, std::string> r;
  const bool remote = std::any_of(nbr_.begin(), nbr_.end(), [&](int n) { return n != a_.rank; });
  const std::string &t = a_.transport;
  if (useRccl_)
    r["rccl"] = rcclGraphOk_ ? (rcclCaptureNote_.empty() ? "ok" : "ok (hipGraph: " + rcclCaptureNote_ + ")")
                             : "ok (eager only: " + rcclGraphWhy_ + ")";
  else if (!rcclWhy_.empty()) r["rccl"] = rcclWhy_;
  else r["rccl"] = "not offered";
  if (useIpc_ && ipcReady_) r["ipc"] = "ok";
  else if (useIpc_) r["ipc"] = ipcWhy_.empty() ? "unavailable" : ipcWhy_;
  else r["ipc"] = "not offered";
  const char *copyNames[2] = {"memcpy_put", "sdma_put"};
  for (int k = 0; k < 2; ++k) {
    if (useIpc_ && ipcReady_ && useCopy_ && !ipcGrid_ && copyOk_[k]) r[copyNames[k]] = "ok";
    else if (!copyWhy_[k].empty()) r[copyNames[k]] = copyWhy_[k];
    else r[copyNames[k]] = "not offered";
  }
  if (uses_wide_puts() && ready()) r["wide_put"] = "ok (" + std::to_string(a_.wide_put_blocks) + " workgroups per box)";
  else if (!wideWhy_.empty()) r["wide_put"] = wideWhy_;
  else r["wide_put"] = "not offered";
  if (uses_relay() && ready()) r["relay"] = "ok";
  else if (relay_) r["relay"] = relayWhy_.empty() ? "unavailable" : relayWhy_;
  else r["relay"] = "not offered";
  if (uses_hostsplit() && ready()) r["hostsplit"] = "ok";
  else if (hsOffered_) r["hostsplit"] = hsWhy_.empty() ? "unavailable" : hsWhy_;
  else r["hostsplit"] = "not offered";
  r["host"] = useHost_ ? "ok" : (remote && (t == "auto" || t == "host") ? "standby" : "not offered");
  return r;
}

bool HaloExchange::bounded_wait(void *stream, double seconds) const {
  const double t0 = wtime();
  hipStream_t s = static_cast<hipStream_t>(stream);
  while (true) {
    const hipError_t r = hipStreamQuery(s);
    if (r == hipSuccess) return true;
    if (r != hipErrorNotReady) TZ_HIP(r);
    if (wtime() - t0 > seconds) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

std::string HaloExchange::rccl_preflight(Ctrl &ctrl) {
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) local.push_back(i);
    else if (pipe_[i]) remote.push_back(i);
  }
  // every rank takes the same steps (the exchanges are collective): whether to run them at all
  // is agreed first
  double none = remote.empty() || comms_.empty() ? 1.0 : 0.0;
  ctrl.allreduce_max(&none, 1);
  if (none != 0.0) return "";
  const double limit = preflight_limit_s(20.0);
  const std::string failEnv = std::getenv("TZ_FAIL_TRANSPORTS") ? std::getenv("TZ_FAIL_TRANSPORTS") : "";
  const bool simHang = ("," + failEnv + ",").find(",rccl_hang,") != std::string::npos;
  const bool simGraph = ("," + failEnv + ",").find(",rccl_graph_schedule,") != std::string::npos;
  hipStream_t s = nullptr, side[2] = {nullptr, nullptr};
  TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (auto &x : side) TZ_HIP(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  std::string why;
  // a hung exchange: release every spinning kernel first (an abort may wait for the device),
  // then abort the communicators on a thread of their own (their kernels return; the abort
  // itself may block), drain the stream with a bound, clear the flag again
  auto hung = [&](const std::string &what) {
    kern::set_abort(true);
    std::vector<std::shared_ptr<RcclComm>> cs = comms_;
    std::thread([cs] {
      for (auto &c : cs)
        if (c && !c->aborted()) c->abort();
    }).detach();
    const bool drained = bounded_wait(s, limit);
    if (!drained)
      // the abort flag cannot be cleared while something still spins, and with it set every
      // device-side wait of every later candidate (IPC arrivals, relays, host split) gives up at
      // once: the search would skip every candidate and measure nothing. End the run with the
      // reason instead (the deadline's partial report says how far it came).
      exit_with_report(6, "RCCL preflight (" + what + "): the device did not drain after the "
                          "communicator abort");
    kern::set_abort(false);
    why = what + " (no completion within " + std::to_string(int(limit)) + " s; communicators aborted)";
  };
  // whatever an error left enqueued must drain, with the same bound
  auto drain_after_error = [&](const std::string &err) {
    bool drained = false;
    try {
      drained = bounded_wait(s, limit);
    } catch (const std::exception &) {
      drained = true; // the stream reports an error: nothing left to wait for
    }
    if (!drained) hung("after an error: " + err);
  };
  // (1) eagerly, one direction at a time, the communicators in turn
  TZ_LOG(Debug, "rccl preflight: eager step, " << remote.size() << " remote direction(s)");
  try {
    if (simHang) kern::busy_wait(int64_t(1) << 50, 1, s); // released by the abort flag
    if (!local.empty()) direct_group(local, s);
    for (size_t k = 0; k < remote.size(); ++k) {
      const int i = remote[k];
      pack(i, s);
      shift(i, s, int(k % comms_.size()));
      unpack(opp_[i], s);
    }
    if (!bounded_wait(s, limit)) {
      hung("per-direction exchange");
    } else if (const uint64_t bad = check_grid(s)) {
      why = "per-direction exchange: " + std::to_string(bad) + " wrong cells";
    }
  } catch (const std::exception &e) {
    why = e.what();
    drain_after_error(why);
  }
  {
    double failed = why.empty() ? 0.0 : 1.0;
    ctrl.allreduce_max(&failed, 1);
    if (failed != 0.0 && why.empty()) why = "failed on another rank";
  }
  // (2) compiled into hipGraphs the way the runtime compiles candidates (GraphBuilder, so RCCL
  // ops take the same capture path): every remote direction in one group, then one RCCL node
  // per direction with the communicators in turn, chained, over three streams of one build.
  // Each graph runs twice, with a new value generation in between: a hang is bounded, and a
  // delivery of the previous launch's data fails the check. Capture modes are tried in turn
  // (whole-schedule capture first), every rank in step; wrong data in one mode moves on to the
  // next, a hang drops RCCL.
  auto graph_step = [&](CaptureMode mode) -> std::string {
    std::string wrong;
    for (int form = 0; form < 2 && why.empty() && wrong.empty(); ++form) {
      hipGraph_t graph = nullptr;
      hipGraphExec_t exec = nullptr;
      try {
        TZ_LOG(Debug, "rccl preflight: graph step, " << capture_mode_name(mode) << " capture, form " << form);
        {
          GraphBuilder gb({s, side[0], side[1]}, mode);
          std::vector<void *> tail = gb.add(0, {}, [&](void *cs) {
            if (!local.empty()) direct_group(local, cs);
            pack_group(remote, cs);
          });
          if (form == 0) {
            tail = gb.add(0, tail, [&](void *cs) { shift_group(remote, cs, 0); });
          } else {
            // as schedules spread them: direction k on stream k % 3 with that stream's
            // communicator (comm_for), chained in one total order like the rccl ordering domain
            for (size_t k = 0; k < remote.size(); ++k) {
              const int si = int(k % 3);
              std::vector<void *> t = gb.add(si, tail, [&](void *cs) { shift(remote[k], cs, si); });
              if (!t.empty()) tail = t;
            }
          }
          gb.add(0, tail, [&](void *cs) { unpack_group(remote, cs); });
          graph = static_cast<hipGraph_t>(gb.finish());
        }
        TZ_LOG(Debug, "rccl preflight: instantiate");
        TZ_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      } catch (const std::exception &e) {
        // a capture or instantiation error is not a broken transport: RCCL stays for eager runs
        wrong = e.what();
        drain_after_error(wrong);
      }
      // launch only where every rank built the graph: a rank launching alone would wait for
      // peers that never join, report a hang and abort the communicators instead of trying the
      // next capture mode
      double built = wrong.empty() ? 0.0 : 1.0;
      ctrl.allreduce_max(&built, 1);
      if (built != 0.0 && wrong.empty()) wrong = "capture or instantiation failed on another rank";
      try {
        TZ_LOG(Debug, "rccl preflight: launch");
        const char *what = form == 0 ? "fused hipGraph exchange" : "per-direction hipGraph exchange";
        const int gens[2][2] = {{1, 2}, {3, 1}}; // (generations are 0..3; 0 is the search's)
        for (int launch = 1; launch <= 2 && why.empty() && wrong.empty(); ++launch) {
          init_grid(s, gens[form][launch - 1]);
          TZ_HIP(hipGraphLaunch(exec, s));
          if (!bounded_wait(s, limit)) {
            hung(what); // communicators aborted: RCCL is gone
          } else {
            uint64_t bad = check_grid(s);
            if (simGraph && mode == CaptureMode::Schedule) bad += 1; // tests: force the fallback
            if (bad)
              wrong = std::string(what) + ", launch " + std::to_string(launch) + ": " +
                      std::to_string(bad) + " wrong cells";
          }
        }
      } catch (const std::exception &e) {
        wrong = e.what();
        drain_after_error(wrong);
      }
      if (exec) (void)hipGraphExecDestroy(exec);
      if (graph) (void)hipGraphDestroy(graph);
      // every rank goes on to the next form (or stops) together
      double f[2] = {why.empty() ? 0.0 : 1.0, wrong.empty() ? 0.0 : 1.0};
      ctrl.allreduce_max(f, 2);
      if (f[0] != 0.0 && why.empty()) why = "failed on another rank";
      if (f[1] != 0.0 && wrong.empty()) wrong = "wrong data on another rank";
    }
    return wrong;
  };
  std::vector<CaptureMode> modes;
  if (capture_mode_forced()) modes = {capture_mode()};
  else modes = {CaptureMode::Schedule, CaptureMode::Child};
  std::vector<std::string> tried;
  bool chosen = false;
  for (size_t m = 0; m < modes.size(); ++m) {
    double flags[2] = {why.empty() ? 0.0 : 1.0, 0.0}; // [failed / hung, wrong data]
    std::string wrong;
    if (flags[0] == 0.0) {
      wrong = graph_step(modes[m]);
      flags[0] = why.empty() ? 0.0 : 1.0;
      flags[1] = wrong.empty() ? 0.0 : 1.0;
    }
    ctrl.allreduce_max(flags, 2);
    if (flags[0] != 0.0) {
      if (why.empty()) why = "failed on another rank";
      break;
    }
    if (flags[1] == 0.0) {
      set_rccl_capture_mode(modes[m]);
      rcclCaptureNote_ = std::string(capture_mode_name(modes[m])) + " capture";
      if (!tried.empty()) rcclCaptureNote_ += " (" + tried.front() + ")";
      chosen = true;
      break;
    }
    tried.push_back(std::string(capture_mode_name(modes[m])) + " capture: " +
                    (wrong.empty() ? "wrong data on another rank" : wrong));
  }
  if (why.empty() && !chosen) {
    // every rank alike: RCCL ops are left out of hipGraphs (candidates with them run eagerly)
    rcclGraphOk_ = false;
    for (const std::string &t : tried) rcclGraphWhy_ += (rcclGraphWhy_.empty() ? "" : "; ") + t;
  }
  (void)hipStreamDestroy(s);
  for (auto &x : side) (void)hipStreamDestroy(x);
  return why;
}

void HaloExchange::init_grid(void *stream, int gen) {
  TZ_CHECK(ready(), "halo not set up");
  TZ_CHECK(gen >= 0 && gen <= 3, "grid generation must be 0..3 (got " << gen << ")");
  gen_ = gen;
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

void HaloExchange::copy_grid(void *ptr, bool toGrid, void *stream) {
  TZ_CHECK(ready(), "halo not set up");
  TZ_CHECK(ptr, "copy_grid: null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t bytes = gridElems_ * sizeof(double);
  if (toGrid) TZ_HIP(hipMemcpyAsync(grid(), ptr, bytes, hipMemcpyDefault, s));
  else TZ_HIP(hipMemcpyAsync(ptr, grid(), bytes, hipMemcpyDefault, s));
  TZ_HIP(hipStreamSynchronize(s));
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
    TZ_CHECK(nbr_[i] == a_.rank, "shift " << dirs_[i].name() << ": the neighbour is remote and RCCL "
                                          "is not in use (host transport: he_hostxfer)");
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
    for (int i : dirs) {
      TZ_CHECK(nbr_[i] == a_.rank, "shift " << dirs_[i].name() << ": the neighbour is remote and "
                                            "RCCL is not in use (host transport: he_hostxfer)");
      cs.push_back({recv_[opp_[i]].get(), send_[i].get(), box_elems(i) * sizeof(double)});
    }
    for (size_t k = 0; k < cs.size(); k += kern::kMaxBoxes)
      kern::copy_many(cs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, cs.size() - k)), stream);
  }
}

std::vector<kern::MoveDesc> HaloExchange::direct_moves(const std::vector<int> &dirs_in) const {
  // faces first, then edges, then corners: blocks are dispatched box by box in batch order,
  // and leaving the many small edge/corner boxes for the last waves measured best (fused
  // 26-direction move 44.13 us vs 44.23 in the natural order and 45.18 with the small boxes
  // first; scripts/box_order_ab.py, profiles/archive/r2_box_order/)
  std::vector<int> dirs = dirs_in;
  std::stable_sort(dirs.begin(), dirs.end(), [&](int a, int b) {
    auto k = [&](int i) { return (dirs_[i].dx != 0) + (dirs_[i].dy != 0) + (dirs_[i].dz != 0); };
    return k(a) < k(b);
  });
  std::vector<kern::MoveDesc> ms;
  for (int i : dirs) {
    TZ_CHECK(i >= 0 && i < ndirs() && direct_[i], "direction " << i << " is not a direct (self) transfer");
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
  if (a_.order == "xyzq" && a_.move_pairs) ms = pair_x_moves(ms);
  return ms;
}

void HaloExchange::direct_group(const std::vector<int> &dirs, void *stream) const {
  TZ_CHECK(ready(), "halo not set up");
  const std::vector<kern::MoveDesc> ms = direct_moves(dirs);
  for (size_t k = 0; k < ms.size(); k += kern::kMaxBoxes)
    kern::box_move_many(ms.data() + k, int(std::min<size_t>(kern::kMaxBoxes, ms.size() - k)), stream);
}

std::map<std::string, double> HaloExchange::move_roof(int iters) {
  // The fused direct move of every self direction against the shape-matched roof: a kernel
  // that touches exactly the lines the move touches (line_boxes: per box, the 128-B lines of
  // its source rows read, of its destination rows written; rows a lane both reads and writes
  // read and written back together), with whole-line 16-B accesses and trivial indexing. Both
  // timed back to back on one stream, `iters` launches each after 3 untimed ones; the grid is
  // initialized again afterwards (the roof writes zeros into the lines it writes).
  TZ_CHECK(ready(), "halo not set up");
  TZ_CHECK(iters >= 1, "iters must be positive");
  std::vector<int> dirs;
  for (int i = 0; i < ndirs(); ++i)
    if (direct_[i]) dirs.push_back(i);
  TZ_CHECK(!dirs.empty(), "move_roof: no direct (self) direction");
  const std::vector<kern::MoveDesc> ms = direct_moves(dirs);
  // the same lines as line-to-line copies where a move's source and target rows cover equal
  // lines (the move's own shape), and as separate read-only and write-only boxes
  const std::vector<kern::LineBox> lb = kern::line_boxes(ms.data(), int(ms.size()), true);
  const std::vector<kern::LineBox> lbSplit = kern::line_boxes(ms.data(), int(ms.size()), false);
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  TZ_HIP(hipEventCreate(&e0));
  TZ_HIP(hipEventCreate(&e1));
  auto time = [&](const std::function<void()> &launch) {
    for (int k = 0; k < 3; ++k) launch();
    TZ_HIP(hipEventRecord(e0, s));
    for (int k = 0; k < iters; ++k) launch();
    TZ_HIP(hipEventRecord(e1, s));
    TZ_HIP(hipEventSynchronize(e1));
    float ms_ = 0;
    TZ_HIP(hipEventElapsedTime(&ms_, e0, e1));
    return double(ms_) * 1e3 / iters;
  };
  std::map<std::string, double> r;
  try {
    r["move_us"] = time([&] { direct_group(dirs, s); });
    // each roof: the fastest of its access variants (items in flight, store policy)
    auto roof = [&](const std::vector<kern::LineBox> &boxes, const std::string &key) {
      double best = 0;
      for (int v = 0; v < kern::kLineRoofVariants; ++v) {
        const double t = time([&] { kern::line_roof(boxes.data(), int(boxes.size()), s, v); });
        r[key + "_v" + std::to_string(v)] = t;
        if (v == 0 || t < best) best = t;
      }
      r[key] = best;
    };
    roof(lb, "roof_us");
    roof(lbSplit, "roof_split_us");
    // the same number of lines read and written as one contiguous line-to-line copy (the plain
    // HBM roof of this traffic, no shape at all)
    int64_t lines = 0;
    for (const kern::LineBox &b : lb)
      if (b.mode != 1) lines += int64_t(b.lines) * b.n1 * b.n2 * b.n3;
    if (lines > 0 && 2 * lines * 16 + (int64_t(1) << 20) <= int64_t(gridElems_) && lines < (int64_t(1) << 27)) {
      kern::LineBox c;
      c.base = c.dst_base = grid();
      c.off = 0;
      c.dst_off = (lines * 16 + (int64_t(1) << 17)) / 16 * 16;
      c.lines = int32_t(lines);
      c.n1 = c.n2 = c.n3 = 1;
      c.mode = 3;
      roof({c}, "copy_roof_us");
    }
    r["move_us_again"] = time([&] { direct_group(dirs, s); });
  } catch (...) {
    (void)hipStreamSynchronize(s);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    throw;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  double rd = 0, wr = 0, payload = 0, rows = 0;
  for (const kern::LineBox &b : lb) {
    const double bytes = 128.0 * b.lines * double(b.n1) * b.n2 * b.n3;
    if (b.mode != 1) rd += bytes;
    if (b.mode != 0) wr += bytes;
  }
  for (int i : dirs) payload += 8.0 * double(box_elems(i));
  for (const kern::MoveDesc &m : ms) rows += double(m.n1) * m.n2 * m.n3;
  r["read_lines_MB"] = rd / 1e6;
  r["write_lines_MB"] = wr / 1e6;
  r["payload_MB"] = payload / 1e6;
  r["line_boxes"] = double(lb.size());
  r["moves"] = double(ms.size());
  r["pairs"] = double(std::count_if(ms.begin(), ms.end(), [](const kern::MoveDesc &m) { return m.pair; }));
  r["lines_TBps_at_roof"] = (rd + wr) / (r["roof_us"] * 1e-6) / 1e12;
  if (r.count("copy_roof_us")) r["lines_TBps_at_copy_roof"] = (rd + wr) / (r["copy_roof_us"] * 1e-6) / 1e12;
  r["lines_TBps_at_move"] = (rd + wr) / (std::min(r["move_us"], r["move_us_again"]) * 1e-6) / 1e12;
  init_grid(nullptr, gen_);
  return r;
}

std::vector<kern::MoveDesc> HaloExchange::pair_x_moves(const std::vector<kern::MoveDesc> &ms) const {
  // XYZQ, x self-wrap: the +x and -x moves of one (dy, dz) cover the same rows, one run at each
  // end of the row. Moved by one lane per row, a row's ghost run and the source run beside it
  // (one 128-B line when x = 0 sits at the row start, as in the reference's layout) are read
  // and written while the line is in L2, instead of by two boxes far apart in time.
  // partner[a] = b: move a (delta < 0) pairs with move b; the pair takes the earlier slot
  std::vector<int> partner(ms.size(), -1);
  std::vector<bool> taken(ms.size(), false);
  for (size_t a = 0; a < ms.size(); ++a) {
    const kern::MoveDesc &m = ms[a];
    const int64_t delta = m.dst_off - m.src_off;
    if (taken[a] || m.src != m.dst || m.len < 1 || m.len > kern::kMaxPairLen || delta >= 0) continue;
    for (size_t b = 0; b < ms.size(); ++b) {
      if (b == a || taken[b]) continue;
      const kern::MoveDesc &q = ms[b];
      if (q.src == m.src && q.dst == m.dst && q.len == m.len && q.n1 == m.n1 && q.n2 == m.n2 &&
          q.n3 == m.n3 && q.s1 == m.s1 && q.s2 == m.s2 && q.s3 == m.s3 &&
          q.src_off == m.src_off + m.len + delta && q.dst_off == m.src_off + m.len) {
        partner[a] = int(b);
        taken[a] = taken[b] = true;
        break;
      }
    }
  }
  std::vector<kern::MoveDesc> out;
  std::vector<bool> done(ms.size(), false);
  for (size_t k = 0; k < ms.size(); ++k) {
    if (done[k]) continue;
    int a = -1;
    if (partner[k] >= 0) a = int(k);
    for (size_t j = 0; j < ms.size() && a < 0; ++j)
      if (partner[j] == int(k)) a = int(j);
    if (a < 0) {
      out.push_back(ms[k]);
      done[k] = true;
      continue;
    }
    kern::MoveDesc p = ms[size_t(a)];
    p.pair = true;
    out.push_back(p);
    done[size_t(a)] = done[size_t(partner[size_t(a)])] = true;
  }
  return out;
}

void HaloExchange::ghost_widening(int ghostDx, int64_t dstOff, int32_t len, int32_t &lead,
                                  int32_t &trail) const {
  // A write of an x ghost run (side -x: ghost-low, +x: ghost-high) covers a few elements less
  // than whole 64-B sectors; the rest of those sectors is row padding (x < 0 or x >= n + 2g),
  // whose contents nobody reads. Widening the rows over that padding turns every x-face write
  // into full-sector writes (a partially written sector costs the memory a read-modify-write).
  // Row strides are multiples of 16 elements, so the alignment of the first row holds for every
  // row.
  lead = trail = 0;
  if (ghostDx == 0 || a_.ghost_align <= 0) return;
  const int64_t rowLen = pitch_; // elements per (y[,q]) row, a multiple of 16
  const int64_t A = a_.ghost_align;
  if (ghostDx < 0) {
    const int64_t x0 = dstOff % rowLen; // ghost-low: padding [0, x0) before it
    const int64_t e = dstOff % A;
    if (e <= x0) lead = int32_t(e);
  } else {
    const int64_t end = dstOff % rowLen + len; // ghost-high: padding [end, rowLen) after
    const int64_t e = (A - (dstOff + len) % A) % A;
    if (end + e <= rowLen) trail = int32_t(e);
  }
}

void HaloExchange::widen_to_sectors(int ghostDx, kern::MoveDesc &m) const {
  int32_t lead = 0, trail = 0;
  ghost_widening(ghostDx, m.dst_off, m.len, lead, trail);
  m.src_off -= lead;
  m.dst_off -= lead;
  m.len += lead + trail;
}

std::vector<int> HaloExchange::pipelined_dirs() const {
  std::vector<int> v;
  for (int i = 0; i < ndirs(); ++i)
    if (!direct_[i]) v.push_back(i);
  return v;
}

void HaloExchange::host_exchange(const std::vector<int> &dirs_in) const {
  // The transport of last resort: device -> host, one control-plane alltoallv, host -> device.
  // Per peer q the payload is my send buffers of every direction d with nbr(d) == q, in
  // direction order; on a periodic grid the receiver r = q expects exactly those directions
  // (nbr_r(-d) == me) in the same order, each into its ghost buffer recv(-d). Runs on the
  // control thread: the synchronizer has made the packs complete before it (an event sync),
  // and the unpacks are issued after it returns.
  TZ_CHECK(ready() && ctrl_, "halo not set up");
  std::vector<int> dirs = dirs_in;
  std::sort(dirs.begin(), dirs.end());
  std::vector<std::string> out(size_t(a_.size));
  for (int i : dirs) {
    check_pipelined(i);
    const size_t bytes = box_elems(i) * sizeof(double);
    std::string &o = out[size_t(nbr_[i])];
    const size_t at = o.size();
    o.resize(at + bytes);
    TZ_HIP(hipMemcpy(&o[at], send_[i].get(), bytes, hipMemcpyDeviceToHost));
  }
  const std::vector<std::string> in = ctrl_->alltoallv(out);
  std::vector<size_t> used(in.size(), 0);
  for (int i : dirs) {
    const int o = opp_[i];
    const size_t from = size_t(nbr_[o]);
    const size_t bytes = box_elems(i) * sizeof(double);
    TZ_CHECK(from < in.size() && used[from] + bytes <= in[from].size(),
             "host exchange: rank " << from << " sent " << in[from].size() << " bytes, fewer than expected");
    TZ_HIP(hipMemcpy(recv_[o].get(), in[from].data() + used[from], bytes, hipMemcpyHostToDevice));
    used[from] += bytes;
  }
  for (size_t r = 0; r < in.size(); ++r)
    TZ_CHECK(used[r] == in[r].size(), "host exchange: rank " << r << " sent " << in[r].size()
                                                              << " bytes, expected " << used[r]);
}

void HaloExchange::pack_all(void *stream) const { pack_group(pipelined_dirs(), stream); }
void HaloExchange::unpack_all(void *stream) const { unpack_group(pipelined_dirs(), stream); }
void HaloExchange::shift_all(void *stream) const { shift_group(pipelined_dirs(), stream); }

} // namespace tz
