// Workload op libraries ("model families"): 3-D halo exchange and distributed CSR SpMV, plus
// small generic GPU ops for user-built graphs.
//
// Parity:
//   halo: include/tenzing/halo_exchange/ops_halo_exchange.hpp:22-186,
//         src/halo_exchange/ops_halo_exchange.cu:33-257 (HaloExchange::add_to_graph, Pack,
//         Unpack, OwningIsend/OwningIrecv, MultiWait), tenzing-mcts/examples/
//         halo_run_strategy.hpp:42-131 (config, rank grid from prime factors, coord maps)
//   spmv: include/tenzing/spmv/ops_spmv.cuh:61-436 (SpMVKernel, Scatter, VectorAdd, PostSend/
//         PostRecv/WaitSend/WaitRecv, SpMV CompoundOp), row_part_spmv.cuh:105-445 (RowPartSpmv),
//         csr_mat.hpp:301-370 (random band matrix), partition.hpp, split_mat.hpp
// MI355X redesign:
//   * halo: per direction d a chain Pack(d) -> Shift(d) -> Unpack(-d). Shift is one grouped
//     RCCL send(S_d -> nbr(d)) + recv(R_-d <- nbr(-d)) on direction d's communicator (the MPI
//     Isend/Irecv/Wait triple of the reference collapses into one stream-ordered op; no host
//     round trip between pack and send). Faces (6) or faces+edges+corners (26, 27-point stencil).
//     Optional fused variants pack/shift/unpack every direction in one op. Single rank: Shift is
//     a device-to-device copy (periodic self-neighbour) unless RCCL is forced.
//     Grid layout is x-padded so interior rows start 64-byte aligned (dwordx4 pack/unpack).
//   * spmv: the matrix is generated deterministically on every rank (no setup communication);
//     the compound op holds Scatter -> Exchange (one grouped RCCL exchange with every peer) ->
//     remote SpMV, local SpMV (a ChoiceOp over lanes-per-row variants), and a real VectorAdd.
#pragma once

#include "core/ctrl.hpp"
#include "core/graph.hpp"
#include "kernels/kernels.hpp"

#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace tz {

class RcclComm;
class RocsparseCsr;

/// the wait bound of a transport preflight (seconds): env TZ_PREFLIGHT_S if set, else `dflt`
/// (RCCL preflight exchanges 20 s, device-side IPC / relay / host-split waits 3 s: a healthy
/// exchange of a preflight's size takes milliseconds)
double preflight_limit_s(double dflt);

/// hipMalloc'd memory (RAII)
class DeviceBuffer {
public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes);
  /// `peerWritten`: another GPU stores into this buffer over xGMI (IPC receive buffers). It is
  /// allocated fine-grained, so the reading kernels see those stores through the caches rather
  /// than lines the local L2 kept from the previous exchange (coarse-grained memory is only
  /// coherent with other agents at dispatch boundaries whose fences the device-side arrival
  /// waits bypass).
  DeviceBuffer(size_t bytes, bool peerWritten);
  ~DeviceBuffer();
  DeviceBuffer(DeviceBuffer &&o) noexcept : p_(o.p_), bytes_(o.bytes_) {
    o.p_ = nullptr;
    o.bytes_ = 0;
  }
  DeviceBuffer &operator=(DeviceBuffer &&o) noexcept;
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;
  void *get() const { return p_; }
  template <typename T> T *as() const { return static_cast<T *>(p_); }
  size_t bytes() const { return bytes_; }
  void upload(const void *src, size_t bytes);
  void download(void *dst, size_t bytes) const;
  /// give the memory up without freeing it (a device that may still be writing into it, e.g.
  /// after a transfer that did not complete in time: freeing would wait for it)
  void leak() {
    p_ = nullptr;
    bytes_ = 0;
  }

private:
  void *p_ = nullptr;
  size_t bytes_ = 0;
};

/// Host memory shared by the processes of one node (POSIX shared memory) and registered with
/// the calling process's GPU (hipHostRegister): this GPU can store into it and another
/// process's GPU can load from it, over each GPU's own PCIe link to the host, beside xGMI. The
/// creator names it; the peers open it by that name; `unlink()` removes the name once everyone
/// has opened it (the mappings stay valid, and nothing is left in /dev/shm).
class SharedHostBuffer {
public:
  SharedHostBuffer() = default;
  /// create (exclusive) and zero-fill `bytes` under `name`; space is reserved up front
  /// (posix_fallocate), so a full /dev/shm fails here and not with SIGBUS on first touch
  static SharedHostBuffer create(const std::string &name, size_t bytes);
  static SharedHostBuffer open(const std::string &name, size_t bytes);
  ~SharedHostBuffer();
  SharedHostBuffer(SharedHostBuffer &&o) noexcept { swap(o); }
  SharedHostBuffer &operator=(SharedHostBuffer &&o) noexcept {
    SharedHostBuffer t(std::move(o));
    swap(t);
    return *this;
  }
  SharedHostBuffer(const SharedHostBuffer &) = delete;
  SharedHostBuffer &operator=(const SharedHostBuffer &) = delete;
  void *host() const { return host_; }
  /// the same bytes as this process's GPU addresses them
  void *dev() const { return dev_; }
  size_t bytes() const { return bytes_; }
  void unlink();

private:
  void swap(SharedHostBuffer &o) noexcept;
  void *host_ = nullptr, *dev_ = nullptr;
  size_t bytes_ = 0;
  std::string name_;
  bool linked_ = false; // this process created the name and has not removed it yet
  bool registered_ = false;
};

// ------------------------------------------------------------------ generic GPU ops

/// launches an empty kernel (reference test/test_gpu_graph.cu KernelOp)
class EmptyKernelOp : public GpuOp {
public:
  explicit EmptyKernelOp(std::string name) : name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "EmptyKernel"; }
  double cost_us() const override { return 2.0; }
  void launch(void *stream, Executor &) const override;

private:
  std::string name_;
};

/// a host function enqueued on the stream (hipLaunchHostFunc; a host node when captured): what
/// RCCL's network proxies add to a captured schedule. Diagnostic op for graph-concurrency probes
class HostFuncOp : public GpuOp {
public:
  explicit HostFuncOp(std::string name) : name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "HostFunc"; }
  double cost_us() const override { return 5.0; }
  void launch(void *stream, Executor &) const override;

private:
  std::string name_;
};

/// a kernel that occupies `blocks` workgroups for `us` microseconds
class BusyKernelOp : public GpuOp {
public:
  BusyKernelOp(std::string name, double us, int blocks = 1)
      : name_(std::move(name)), us_(us), blocks_(blocks) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "BusyKernel"; }
  double cost_us() const override { return us_; }
  Json json() const override;
  void launch(void *stream, Executor &) const override;

private:
  std::string name_;
  double us_;
  int blocks_;
};

/// This machine, as a fixed-size string (host name and boot id): the IPC transports exchange it
/// with their handles and map a peer's memory only when the peer runs on the same node. A
/// handle from another node must never be opened.
constexpr size_t kNodeIdBytes = 96;
std::string node_identity();

/// All-pairs link probe (link_matrix.cpp): put[r][q] / sdma[r][q] = GB/s rank r moved into rank
/// q's IPC-mapped buffer by the halo's kernel put / the SDMA engines, every rank sending at once
/// (round s: r -> (r + s) % P); -1 where not measured; `why` says why nothing was ("" = ok)
struct LinkMatrix {
  std::vector<std::vector<double>> put, sdma;
  double bytes = 0;
  int iters = 0;
  std::string why;
  bool stuck = false; // a transfer did not complete within the wait limit (on some rank)
};
/// collective over `ctrl`: `bytes` per transfer (a multiple of 32 KiB), `iters` per round; every
/// device wait gives up after `wait_limit_s` (the result then says why, and `stuck` is set)
LinkMatrix link_matrix(Ctrl &ctrl, size_t bytes, int iters, double wait_limit_s = 30.0);

// ------------------------------------------------------------------ halo exchange

struct HaloArgs {
  int nx = 512, ny = 512, nz = 512, nq = 3, ghost = 3;
  int neighbors = 6;              // 6 (faces) or 26 (faces, edges, corners)
  std::string order = "xyzq";     // "xyzq" (x fastest, q slowest) or "qxyz"
  // "rccl" (pack -> grouped RCCL send/recv -> unpack), "copy" (pack -> device copy -> unpack,
  // self-neighbours only), "direct" (pack-free box moves straight into the neighbour's ghost
  // region; self-neighbours only), "ipc" (self-neighbours direct; remote directions are
  // pack-free puts into the peer's IPC-mapped grid plus a device-side arrival wait — also the
  // loopback backend for several ranks on one GPU), "auto" (direct on one rank, direct + rccl
  // otherwise), "host" (pack -> device-to-host copy -> control-plane exchange -> host-to-device
  // copy -> unpack: slow but available whenever the control plane is; "auto" falls back to it
  // when neither RCCL nor IPC passes its preflight)
  std::string transport = "auto";
  // "choice": per group (faces / edges+corners) the search chooses per-direction or fused ops;
  // "none": per-direction ops; "groups": fused per group; "pack": fused pack+unpack with
  // per-direction transfers; "all": one op per stage
  std::string fuse = "choice";
  // RCCL communicators (0 = kDefaultComms). A transfer uses the communicator of the logical
  // stream it runs on, so transfers on different streams never share one (RCCL serializes
  // operations of one communicator) and a whole exchange needs only a few communicators
  int comms = 0;
  int rank = 0, size = 1;
  int px = 0, py = 0, pz = 0;     // rank grid (0 = from prime factors, reference style)
  int pitch_pad = 0;              // extra row-pitch elements (multiple of 8; of 16 with ghost_align 16)
  // 8 or 16: the x padding puts the inner ends of the x ghost runs (ghost-low end, ghost-high
  // start) on 8-element (64-B sector) / 16-element (128-B line) boundaries, and direct moves
  // widen their x ghost writes over the neighbouring row padding to whole sectors / lines (no
  // partially written sectors or lines on the x faces). 0: line-optimal padding, exact runs.
  // -1: no padding, x = 0 at the row start (the reference's layout). -2 (default): 16.
  int ghost_align = -2;
  // IPC puts land in the peer's grid (1) or in receive buffers that the peer unpacks (0);
  // -1 (default): the grid below 2 GiB (measured, scripts/ipc_probe.py), buffers above
  int ipc_grid = -1;
  // copy-engine puts (SDMA, hipMemcpy) offered beside the kernel puts (buffers mode only)
  bool copy_puts = true;
  // copy-engine puts of one group spread over this many streams (1..8): one engine moves
  // ~60 GB/s, independent copies on 2 / 4 streams reach more on one device
  int copy_engines = 1;
  // XYZQ self-wrap moves of the x axis as row pairs (one lane moves a row's +x and -x runs,
  // which share lines in the row-start layout); false: separate moves (A/B)
  bool move_pairs = true;
  // grid memory: -1 auto (fine-grained when peers store into it, i.e. IPC "grid" mode; else
  // coarse-grained), 0 coarse-grained, 1 fine-grained. A peer's stores over xGMI bypass this
  // GPU's L2, so a coarse-grained grid may keep stale or dirty lines of the ghost cells
  int grid_memory = -1;
  // appended to this process's node identity (tests: ranks on one node posing as several
  // nodes). Directions whose neighbour is on another node go over RCCL (see HaloExchange)
  std::string node_tag;
  // also run a 7-point stencil over the interior after the exchange (into a second grid): the
  // search may update the ghost-free interior while ghosts are in flight and the one-cell
  // boundary shell afterwards, or the whole domain after the exchange (a ChoiceOp)
  bool stencil = false;
  // two-hop routing of part of every face through the corner peer (2x2x2 rank grid, IPC
  // "buffers" mode). Each GPU has one xGMI link per peer, and in a 2x2x2 grid both faces of an
  // axis go to the same peer, so the 3 face links carry almost all bytes while the 3
  // edge-diagonal links and the corner link idle. A relayed share f of each face goes
  // r -> r+(1,1,1) (corner link) -> r+d (that rank's edge-diagonal link): every link then
  // carries at most 0.75 of a face pair for f = 0.25 with overlapped forwarding, or 0.8 for
  // f = 0.2 with forwarding after arrival (what is built). "auto": offered to the search as a
  // transport alternative when applicable; "off"; "force": the only remote transport (tests)
  std::string relay = "auto";
  std::vector<double> relay_fracs = {0.15, 0.2, 0.25}; // relayed shares offered (a ChoiceOp; 0.25: f* at equal link rates)
  // host split (IPC "buffers" mode, several ranks): a share of every face goes GPU -> node
  // shared host memory -> peer GPU over each GPU's own PCIe link, while the rest goes over
  // xGMI as an IPC put; the PCIe links are otherwise idle during an exchange. "auto": offered
  // to the search when its preflight passes; "off"; "force": the only remote transport (tests)
  std::string hostsplit = "auto";
  std::vector<double> hostsplit_fracs = {0.1, 0.2, 0.3, 0.4}; // host shares offered (a ChoiceOp)
  // the host share of a face travels in this many chunks, each signalled on its own, so the
  // receiver's DMA of one chunk can overlap the sender's PCIe stores of the next. Default 1 (all
  // stores, then one DMA): 4 chunks measured 7-17 % slower on 2 loopback ranks, whose PCIe
  // link sees the same store / read-back mix as one GPU's link on a node (profiles/archive/r3_hs_chunks)
  int hostsplit_chunks = 1;
  // wide kernel puts: the IPC put kernels with `wide_put_blocks` workgroups per box instead of
  // the global cap (BoxTuning::put_max_blocks, 64), offered to the search as a transport alternative.
  // One loopback GPU has no link to fill, so 64 won there; whether more workgroups in flight
  // fill an xGMI link better is the node's to measure. "auto": offered when a peer's memory
  // sits on another device (agreed by every rank); "on": always (tests); "off"
  std::string wide_puts = "auto";
  int wide_put_blocks = 256;
  int device = -1;
  Json json() const;
};

class HaloExchange : public std::enable_shared_from_this<HaloExchange> {
public:
  struct Dir {
    int dx, dy, dz;
    std::string name() const;
  };

  explicit HaloExchange(HaloArgs a);
  ~HaloExchange();

  const HaloArgs &args() const { return a_; }
  int ndirs() const { return int(dirs_.size()); }
  const Dir &dir(int i) const { return dirs_[i]; }
  int opposite(int i) const { return opp_[i]; }
  int neighbor(int i) const { return nbr_[i]; }
  std::array<int, 3> coords() const { return {cx_, cy_, cz_}; }
  std::array<int, 3> rank_grid() const { return {a_.px, a_.py, a_.pz}; }
  int coord_to_rank(int x, int y, int z) const;
  kern::BoxDesc pack_box(int i) const;   // interior slab facing direction i (buf filled later)
  kern::BoxDesc unpack_box(int i) const; // ghost region on side i
  size_t box_elems(int i) const;
  size_t grid_elems() const { return gridElems_; }
  double exchange_bytes() const; // bytes sent per exchange by this rank
  kern::HaloGeom geom() const;

  /// allocate device memory and (for RCCL) communicators; collective over ctrl when size > 1
  void setup(Ctrl *ctrl);
  bool ready() const { return grid_.get() != nullptr; }
  /// add the exchange's ops and edges to g (Start -> packs ... unpacks -> Finish); in stencil
  /// mode the stencil around it
  void add_to_graph(Graph &g);
  /// the exchange alone
  void add_exchange(Graph &g);

  // device data
  double *grid() const { return grid_.as<double>(); }
  /// interior = encoded global coordinates of generation `gen` (0..3), ghosts = -1; the checks
  /// below expect the values of the last initialized generation
  void init_grid(void *stream = nullptr, int gen = 0);
  /// number of wrong elements after an exchange (0 = all ghosts correct, interior untouched)
  uint64_t check_grid(void *stream = nullptr);
  /// copy the whole grid storage (grid_elems() doubles) to `ptr` (toGrid false) or from it
  /// (toGrid true); any device or host pointer; synchronous. Lets a test check an exchange
  /// against an independent model of the layout instead of check_grid's own formula
  void copy_grid(void *ptr, bool toGrid, void *stream = nullptr);
  /// stencil mode: number of output cells that differ from the stencil of the initialized grid
  uint64_t check_stencil(void *stream = nullptr);
  /// stencil mode: apply the stencil to an interior region: 0 = ghost-free interior
  /// [1, n-1)^3, 1 = the one-cell boundary shell, 2 = the whole interior
  void stencil(int region, void *stream) const;
  double *stencil_out() const { return out_.as<double>(); }

  // op bodies
  void pack(int i, void *stream) const;
  void unpack(int i, void *stream) const;
  /// `streamIdx`: the executor's logical stream (selects the RCCL communicator; -1: by direction)
  void shift(int i, void *stream, int streamIdx = -1) const;
  void pack_all(void *stream) const;
  void unpack_all(void *stream) const;
  void shift_all(void *stream) const;
  /// one launch / one RCCL group for a set of directions (unpack: their opposite ghosts)
  void pack_group(const std::vector<int> &dirs, void *stream) const;
  void unpack_group(const std::vector<int> &dirs, void *stream) const;
  void shift_group(const std::vector<int> &dirs, void *stream, int streamIdx = -1) const;
  std::vector<int> all_dirs() const;
  /// directions that go through pack -> transfer -> unpack (not direct)
  std::vector<int> pipelined_dirs() const;
  /// k = 1 faces, 2 edges, 3 corners, 0 edges + corners
  std::vector<int> group_dirs(int k) const;
  bool uses_rccl() const { return useRccl_; }
  /// RCCL exchanges passed the hipGraph part of the preflight (else RCCL ops run eagerly only)
  bool rccl_graph_ok() const { return rcclGraphOk_; }
  bool uses_direct() const { return useDirect_; }
  bool uses_ipc() const { return useIpc_; }
  /// the host-staged transport carries the remote directions (no device transport works)
  bool uses_host() const { return useHost_; }
  /// ranks of the RCCL communicators after setup (0: RCCL not in use)
  int rccl_nranks() const;
  /// per transport ("rccl", "ipc", "relay", "host"): "ok", "not offered", or why it is
  /// unavailable (creation or preflight failure), after setup
  std::map<std::string, std::string> transport_report() const;
  /// for every peer rank whose memory this rank mapped over IPC: the device the mapped flags
  /// allocation reports (hipPointerGetAttributes), -1 if that query fails. On a multi-GPU node
  /// a peer's memory must sit on another device than this rank's; on loopback, on the same one.
  std::map<int, int> ipc_peer_devices() const;
  /// collective, every rank idle: restart the IPC put / wait counters (and clear the wait
  /// timeouts) from zero, e.g. after a verification run that timed out; a barrier otherwise
  void reset_transport_state(Ctrl *ctrl) {
    if (useIpc_ && ipcReady_) reset_ipc_counters(ctrl);
    else ctrl->barrier();
  }
  /// host-staged transport: every rank's send buffers of `dirs` to their neighbours through the
  /// control plane (one alltoallv), into the receive buffers of the opposite ghosts
  void host_exchange(const std::vector<int> &dirs) const;
  /// direction i is moved directly (self-neighbour) rather than packed and transferred
  bool is_direct(int i) const { return direct_[i]; }
  /// direction i is a pack-free put into the neighbour's IPC-mapped grid
  bool is_ipc(int i) const { return ipc_[i]; }
  /// available transports joined by "+": "direct" (self-neighbour moves), "rccl", "ipc"
  /// (when both rccl and ipc are listed the search chooses), or "copy"
  std::string transport() const {
    std::string t;
    auto add = [&](const char *x) { t += (t.empty() ? "" : "+") + std::string(x); };
    if (useDirect_) add("direct");
    if (useRccl_) add("rccl");
    if (useIpc_ && (ipcReady_ || !ready())) add("ipc");
    if (useHost_) add("host");
    return t.empty() ? "copy" : t;
  }
  /// ipc transport: put my slabs facing `dirs` into the neighbours' ghost regions and signal
  /// their arrival counters (one launch)
  /// (`max_blocks`: workgroups per box at most, 0 = the global cap)
  void put_group(const std::vector<int> &dirs, void *stream, int max_blocks = 0) const;
  /// ipc transport, copy-engine variant ("buffers" mode): pack locally, hipMemcpyAsync into the
  /// neighbours' receive buffers, then signal their arrival counters. `sdma`: force the SDMA
  /// engines (no CUs); otherwise the runtime picks the copy engine
  void copy_put_group(const std::vector<int> &dirs, void *stream, bool sdma = true) const;
  /// ipc transport: wait until the ghosts filled by the neighbours' puts of `dirs` arrived
  void wait_group(const std::vector<int> &dirs, void *stream) const;
  /// ipc "buffers" mode: unpack the receive buffers filled for `dirs`, then return the
  /// senders' credits (their next put may overwrite the buffers)
  void ipc_unpack_group(const std::vector<int> &dirs, void *stream) const;
  /// ipc transport: number of arrival waits that timed out (0 = healthy); resets the flag
  int ipc_errors();
  /// ipc transport: "grid" (puts land directly in the peer's ghost cells) or "buffers" (puts
  /// fill the peer's receive buffers, which it unpacks after the arrival wait). Grids of 2 GiB
  /// or more use "buffers": the dmabuf IPC path of this platform cannot map allocations that
  /// large (measured, scripts/ipc_probe.py); env TZ_IPC_GRID=0/1 forces a mode. Grid mode
  /// returns each credit right after the arrival, so ghosts stay valid only until the peer's
  /// next put: stencil mode (which reads them after the exchange) always uses "buffers".
  std::string ipc_mode() const { return useIpc_ ? (ipcGrid_ ? "grid" : "buffers") : ""; }
  /// "fine" or "coarse": the grid's memory (set up)
  std::string grid_memory() const { return gridFine_ ? "fine" : "coarse"; }
  /// relay routing (see HaloArgs::relay) is available: rank grid 2x2x2, ipc buffers mode
  bool uses_relay() const { return relay_ && useIpc_ && (relayReady_ || !ready()); }
  /// remote directions whose neighbour runs on another node (on some rank: the split is the
  /// same on every rank); they go over RCCL while the others keep the IPC transports
  /// the off-node directions' exchange over RCCL (pack, shift, unpack), collective
  void off_node_exchange(void *stream) const;
  std::vector<int> off_node_dirs() const {
    std::vector<int> v;
    for (int i = 0; i < int(offNode_.size()); ++i)
      if (offNode_[size_t(i)]) v.push_back(i);
    return v;
  }
  /// relay routing, direct link: put the first (1 - f) share of every face of `faces` and the
  /// whole box of every other direction of `dirs` into the neighbours' receive buffers
  void relay_put_direct(const std::vector<int> &dirs, double frac, void *stream) const;
  /// relay routing, first hop: put the last share f of every face of `faces` into the corner
  /// peer's relay buffers (one launch, arrival signals in its relay slots)
  void relay_put_corner(const std::vector<int> &faces, double frac, void *stream) const;
  /// relay routing, second hop: wait for my corner-origin's relayed shares, copy them into
  /// their final receivers' receive buffers behind the direct share, signal those receivers and
  /// return the relay credits to the origin. `sdma`: the copies run on the copy engines
  /// (hipMemcpyAsync) instead of a kernel, leaving the CUs to the concurrent direct put
  void relay_forward(const std::vector<int> &faces, double frac, void *stream, bool sdma = false) const;
  /// relay routing: wait for every direct put of `dirs` and every forwarded share of `faces`
  void relay_wait(const std::vector<int> &dirs, const std::vector<int> &faces, void *stream) const;
  /// relay routing: unpack `dirs` (faces as direct + relayed sub-boxes) and return the credits
  /// of the direct senders and of the forwarders
  void relay_unpack(const std::vector<int> &dirs, const std::vector<int> &faces, double frac,
                    void *stream) const;
  /// wide kernel puts (see HaloArgs::wide_puts) are offered: agreed and preflighted at setup;
  /// for graph-only builds when wide_puts is "on"
  bool uses_wide_puts() const {
    return useIpc_ && (ready() ? ipcReady_ && widePuts_ : a_.wide_puts == "on");
  }
  /// this rank's wide-put offer (before the agreement, which takes the max over ranks): "on"
  /// always, "off" never, "auto" when a peer of an IPC direction has another PCI bus id than
  /// mine, or the runtime maps a peer's memory on another device than mine (empty bus ids and
  /// negative devices are unknown and decide nothing)
  static bool wide_puts_offered(const std::string &mode, const std::string &myBus,
                                const std::vector<std::string> &peerBuses, int myDevice,
                                const std::vector<int> &mappedDevices);
  /// the face directions among the remote ones (what relay routing splits)
  std::vector<int> relay_faces() const;
  /// host split (HaloArgs::hostsplit) is available: ipc buffers mode, shared host memory mapped
  bool uses_hostsplit() const { return hsOffered_ && useIpc_ && (hsReady_ || !ready()); }
  /// host split: the first (1 - f) share of every face of `dirs` (and every other direction
  /// whole) as IPC puts into the neighbours' receive buffers (relay routing's direct put)
  void split_put_direct(const std::vector<int> &dirs, double frac, void *stream) const;
  /// host split: the last share f of every face of `faces` into the receivers' shared host
  /// memory (kernel stores over PCIe), chunk by chunk (HaloArgs::hostsplit_chunks, one launch
  /// each), every chunk followed by its host arrival flag (single-writer stores)
  void hs_put_host(const std::vector<int> &faces, double frac, void *stream) const;
  /// host split: wait for the IPC puts of `dirs` (the host chunks are waited for one by one in
  /// hs_unpack, so their DMAs overlap the sender's later chunks)
  void hs_wait(const std::vector<int> &dirs, const std::vector<int> &faces, void *stream) const;
  /// host split: unpack the IPC shares and return their credits; then per chunk wait for its
  /// arrival and DMA it from host memory behind the direct share; return the host credits and
  /// unpack the host shares
  void hs_unpack(const std::vector<int> &dirs, const std::vector<int> &faces, double frac,
                 void *stream) const;
  /// box `b` cut into at most `parts` sub-boxes along its largest dimension (slower on ties),
  /// in order; their buffers (when b.buf is set) follow one another from b.buf, each on a 128-B
  /// boundary
  static std::vector<kern::BoxDesc> chunk_box(const kern::BoxDesc &b, int parts);
  /// host split: chunks per face of share `frac` (at most hostsplit_chunks; the same for every
  /// face, so that each chunk launch holds every face)
  int hs_parts(double frac) const;
  /// Link probe (collective): every rank moves its slab facing direction `dir` to its
  /// neighbour there, `iters` times, through `via` ("put": kernel stores into the peer's
  /// memory, "put_wide": the same with HaloArgs::wide_put_blocks workgroups per box,
  /// "put_cap<N>": with N workgroups per box, "sdma":
  /// copy engines, "rccl": pack + RCCL send/recv + unpack), one transfer at a
  /// time on one stream. Each transfer crosses one xGMI link per rank, so this measures what one
  /// link carries with that transport. "pair_put" / "pair_sdma" / "pair_mixed" move both faces
  /// of the axis at once (kernel puts, copy engines, or the + face by kernel and the - face by
  /// copy engines on two streams): with 2 ranks along the axis both cross the same link.
  /// Returns seconds per transfer, max over ranks.
  double link_probe(int dir, const std::string &via, int iters, Ctrl *ctrl);
  /// direct transport: move the interior slab facing each direction of `dirs` straight into
  /// the neighbour's ghost region on the opposite side (one launch)
  void direct_group(const std::vector<int> &dirs, void *stream) const;
  /// the moves of direct_group (order, widening, row pairs), not launched
  std::vector<kern::MoveDesc> direct_moves(const std::vector<int> &dirs) const;
  /// the fused direct move of every self direction against its shape-matched roof (a kernel
  /// touching exactly the same 128-B lines with whole-line accesses): microseconds per launch
  /// of both, the lines read / written (MB) and the payload; re-initializes the grid
  std::map<std::string, double> move_roof(int iters);
  void direct(int i, void *stream) const { direct_group({i}, stream); }

private:
  // graph builders; remote directions go through `via`: pack/transfer/unpack (kViaPipe), IPC
  // puts (kViaPut), copy-engine puts on the SDMA engines (kViaCopy) or with the runtime's copy
  // engine (kViaMemcpy), wide kernel puts (kViaPutWide)
  static constexpr int kViaPipe = 0, kViaPut = 1, kViaCopy = 2, kViaMemcpy = 3, kViaPutWide = 4;
  void add_chains(Graph &g, const std::vector<int> &dirs, int via);
  void add_fused(Graph &g, const std::vector<int> &dirs, const std::string &tag, int via);
  void add_structure(Graph &g, const std::vector<int> &dirs, int via,
                     const std::string &pre, const std::string &tagPre = ""); // fuse mode over `dirs`
  void add_ipc_part(Graph &g, const std::vector<int> &remote, int via);
  void add_relay_part(Graph &g, const std::vector<int> &remote, double frac);
  /// buffers mode: the two faces of every axis go to their peers by different engines at once
  /// (positive side: kernel puts, negative side: copy-engine puts; edges and corners: kernel)
  void add_mixed_part(Graph &g, const std::vector<int> &remote);
  void add_hostsplit_part(Graph &g, const std::vector<int> &remote, double frac);
  std::string setup_hostsplit(Ctrl *ctrl); // collective; "" on success
  void hostsplit_preflight(Ctrl *ctrl);    // one verified exchange per share, collective
  void reset_ipc_counters(Ctrl *ctrl);     // every rank idle: all put / wait counters to 0
  int recoveryHook_ = 0; // health.hpp recovery hook (reset_ipc_counters), 0 = none
  bool hsOffered_ = false, hsReady_ = false;
  std::string hsWhy_;
  int hsChunks_ = 1;                    // HaloArgs::hostsplit_chunks
  int gen_ = 0;                         // init_grid's generation
  // my inbox: [arrivals chunks x nd | credits nd | share regions]
  SharedHostBuffer hsMine_;
  std::vector<SharedHostBuffer> hsPeer_; // per rank: its inbox, mapped here (neighbours only)
  std::vector<size_t> hsRegion_;        // per ghost side: byte offset of its region in an inbox
  // [expected arrivals chunks x nd | expected credits nd | arrival counts chunks x nd |
  //  credit counts nd]
  DeviceBuffer hsBook_;
  void check_pipelined(int i) const;
  std::string setup_ipc(Ctrl *ctrl); // "" on success, else why IPC cannot be used
  void ipc_preflight(Ctrl *ctrl);    // one verified exchange; disables IPC collectively on failure
  /// verified RCCL exchanges before the search may use RCCL: every direction on its own (each
  /// communicator in turn) eagerly, then one fused group compiled into a hipGraph, each under a
  /// bounded wait (a hang aborts the communicators instead of blocking). "" on success
  /// collective: the verified RCCL exchanges (eager, then hipGraphs in each capture mode until
  /// one is exact on every rank); returns why RCCL must be dropped ("" = it stays)
  std::string rccl_preflight(Ctrl &ctrl);
  /// wait for `stream` up to `seconds`; false on timeout (the caller aborts)
  bool bounded_wait(void *stream, double seconds) const;
  void drop_rccl(const std::string &why); // RCCL unavailable: abort and release communicators
  std::string rcclWhy_, ipcWhy_;
  bool rcclGraphOk_ = true;
  std::string rcclGraphWhy_; // why RCCL ops are not captured into hipGraphs ("" = they are)
  std::string rcclCaptureNote_; // which capture mode the graph preflight settled on, and why
  bool useHost_ = false;
  Ctrl *ctrl_ = nullptr; // the control plane of setup (host transport)
  HaloArgs a_;
  std::vector<Dir> dirs_;
  std::vector<int> opp_, nbr_;
  int cx_ = 0, cy_ = 0, cz_ = 0;
  int64_t xoff_ = 0, pitch_ = 0, sy_ = 0, sz_ = 0, sq_ = 0;
  size_t gridElems_ = 0;
  bool useRccl_ = false, useDirect_ = false, useIpc_ = false;
  std::vector<bool> direct_, ipc_, pipe_; // per direction: self move / IPC put / pack-transfer-unpack
  bool ipcReady_ = false;
  bool useCopy_ = false; // copy-engine puts offered (buffers mode)
  // copy-engine put variants that passed copy_preflight: [0] runtime-chosen engine
  // (hipMemcpyDeviceToDevice), [1] forced SDMA engines; a failed variant is no longer offered
  bool copyOk_[2] = {true, true};
  std::string copyWhy_[2];
  /// one verified exchange per copy-engine put variant before the search may use it (the
  /// kernel-put preflight does not exercise the copy engines' peer path); collective
  void copy_preflight(Ctrl *ctrl);
  // wide kernel puts: offered (HaloArgs::wide_puts, agreed) and their preflight passed
  bool widePuts_ = false;
  std::string wideWhy_;
  /// decide whether wide puts are offered (collective) and verify them with one exchange of
  /// their own; a failure drops only that variant
  void wide_put_preflight(Ctrl *ctrl);
  // copy-engine puts can spread every copy over this many streams (one SDMA engine each; env
  // HaloArgs::copy_engines). One engine moves ~60 GB/s, and independent copies on 2 / 4 streams reach
  // 120 / 235 GB/s. Forking the chunks from the op's stream and joining them back through events
  // costs more than it gains (19 MB: 58 GB/s on one stream, 33 on two, 15 on four;
  // scripts/sdma_probe.hip, profiles/archive/r2_sdma/), so the default keeps one stream per op and
  // leaves engine parallelism to the search (per-direction copy ops on different streams).
  int copyEngines_ = 1;
  struct EngineSet {
    std::vector<void *> streams; // engines 1.. (engine 0 is the op's stream)
    std::vector<void *> events;  // fork + one join per extra engine
  };
  mutable std::mutex enginesMu_;
  mutable std::map<void *, EngineSet> engines_; // per schedule stream (engines_for)
  EngineSet &engines_for(void *stream) const;
  struct Copy {
    void *dst;
    const void *src;
    size_t bytes;
  };
  /// issue `copies` on the copy engines behind everything already on `stream`, and make
  /// `stream` wait for all of them (fork / join through events; captures into hipGraphs).
  /// `sdma`: hipMemcpyDeviceToDeviceNoCU, else hipMemcpyDeviceToDevice
  void engine_copies(const std::vector<Copy> &copies, void *stream, bool sdma = true) const;
  // ipc transport state
  // counters per direction, uncached and IPC-exported, in kSlotSets sections of ndirs():
  // arrivals | credits | relay arrivals | relay credits | forwarded arrivals | forward credits
  void *flags_ = nullptr;
  static constexpr int kSlotSets = 6;
  DeviceBuffer expected_, done_, err_;
  DeviceBuffer sent_; // per direction: puts issued so far (credit wait bookkeeping)
  // relay bookkeeping: relay arrivals expected | relay puts issued | forwarded arrivals
  // expected | forwards issued (4 x ndirs())
  DeviceBuffer relayBook_;
  bool relay_ = false, relayReady_ = false;
  std::string relayWhy_; // why this rank could not map the relay peers ("" = fine)
  int corner_ = -1;                          // r + (1,1,1): where my relayed shares go
  std::vector<DeviceBuffer> relayBuf_;       // per face direction: shares relayed through me
  std::vector<void *> peerRelay_;            // per face direction: the corner peer's relay buffer
  std::vector<void *> peerFwdRecv_;          // per face direction: final receiver's buffer
  std::vector<int> fwdTo_, fwdFrom_;         // per direction: rank I forward to / forwards to me
  int relayOrigin_ = -1;                     // r - (1,1,1): whose shares I forward
  /// split a box (and its dense buffer) into the direct share A and the relayed share B along
  /// its largest dimension; B holds round(frac * n) rows (at least 1)
  void split_box(const kern::BoxDesc &b, double frac, kern::BoxDesc &A, kern::BoxDesc &B) const;
  void relay_preflight(Ctrl *ctrl);
  unsigned long long *peer_slot(int rank, int set, int i) const;
  std::vector<unsigned long long *> credit_ptrs(const std::vector<int> &dirs) const;
  const RcclComm &comm_for(int streamIdx, int dir) const;
  /// XYZQ direct moves: the +x / -x moves of one (dy, dz) as one row-pair move
  /// (HaloArgs::move_pairs)
  std::vector<kern::MoveDesc> pair_x_moves(const std::vector<kern::MoveDesc> &ms) const;
  void widen_to_sectors(int ghostDx, kern::MoveDesc &m) const;
  /// elements of row padding an x ghost run's writes may also cover before / after each row
  /// (whole ghost_align units); 0, 0 for other boxes or without line-aligned ghosts
  void ghost_widening(int ghostDx, int64_t dstOff, int32_t len, int32_t &lead, int32_t &trail) const;
  static constexpr int kDefaultComms = 4;
  bool ipcGrid_ = true;
  bool gridFine_ = false; // the grid is fine-grained memory (HaloArgs::grid_memory)
  // directions whose neighbour (on some rank) runs on another node: RCCL only, beside IPC for
  // the rest (set up by node identity; empty on one node)
  std::vector<char> offNode_;
  std::vector<void *> peerGrid_, peerFlags_; // per rank (nullptr: not a neighbour / self)
  std::vector<void *> peerRecv_;             // per direction: the receiver's buffer ("buffers")
  std::vector<void *> opened_;               // IPC mappings to close
  double ipcTimeoutS_ = 10.0;                // arrival wait limit (env TZ_IPC_TIMEOUT)
  DeviceBuffer grid_;
  std::vector<DeviceBuffer> send_, recv_;
  std::vector<std::shared_ptr<RcclComm>> comms_;
  DeviceBuffer count_;
  DeviceBuffer out_; // stencil output grid (stencil mode)
  kern::StencilBox stencil_box(int x0, int x1, int y0, int y1, int z0, int z1) const;
};

// ------------------------------------------------------------------ distributed SpMV

struct CsrHost {
  int64_t rows = 0, cols = 0;
  std::vector<int32_t> rowPtr, colInd;
  std::vector<float> val;
  int64_t nnz() const { return int64_t(colInd.size()); }
};

/// deterministic random band matrix: `nnz` entries with |row - col| < bw, values in [-1,1)
/// (reference csr_mat.hpp:334-370 uses rand() and all-ones values)
CsrHost random_band_matrix(int64_t n, int64_t bw, int64_t nnz, uint64_t seed);
/// Matrix Market coordinate file -> CSR (real / integer / pattern values; general, symmetric
/// or skew-symmetric storage; 1-based indices; duplicate entries summed). The reference vendors
/// an MTX reader (thirdparty/cwpearson/mm) but never calls it; here the SpMV workload can run
/// on any square matrix from a file (SpmvArgs::matrix).
CsrHost read_matrix_market(const std::string &path);
/// write A as "matrix coordinate real general" (round trips through read_matrix_market)
void write_matrix_market(const CsrHost &A, const std::string &path);
/// rows [r0, r1) owned by rank (remainder to low ranks, reference partition.hpp:21-76)
std::pair<int64_t, int64_t> row_partition(int64_t n, int rank, int size);

struct SpmvArgs {
  // Matrix Market file of a square matrix to use instead of the random band matrix ("" = the
  // reference's random band matrix of m rows); every rank reads it (no setup communication)
  std::string matrix = "";
  int64_t m = 150000;
  int64_t bw = 0;  // 0 = m / size (reference spmv_run_strategy.cuh:67)
  int64_t nnz = 0; // 0 = 10 * m
  int64_t nnz_actual = 0; // set by DistSpmv: the entries of the matrix it built or read
  uint64_t seed = 1;
  int rank = 0, size = 1;
  int device = -1;
  bool compound = true;     // wrap in an expandable CompoundOp (reference SpMV CompoundOp)
  bool kernel_choice = true; // local SpMV as a ChoiceOp over lanes-per-row variants
  // rocSPARSE CSR algorithm added to that ChoiceOp as a library comparison variant (the
  // reference's cuSPARSE SpMV); "" leaves the library out
  std::string library = "adaptive";
  // "split": y = A_l x + A_r x_r through two partial vectors and a VectorAdd (reference
  // structure); "accum": y = A_l x, then y += A_r x_r (no partials, no add; the remote SpMV
  // waits for the local one); "choice": a ChoiceOp over both forms
  std::string form = "choice";
  // x-halo transport between ranks: "rccl" (gather -> grouped RCCL exchange), "ipc" (the gather
  // kernel stores straight into the peers' IPC-mapped remote-x buffers + device-side arrival
  // wait; also the loopback backend for several ranks on one GPU), "auto" (both as a ChoiceOp
  // when both can be set up, else whichever can)
  std::string transport = "auto";
  std::string prefix = "";  // op-name prefix (to combine several workloads in one graph)
  // "root": rank 0 builds / reads the matrix and sends every rank its rows, then each rank asks
  // the owners for the x entries it needs (the reference's setup); "local": every rank builds
  // the whole matrix and derives every plan itself (no setup messages); "auto": root when the
  // control plane is given and there are several ranks
  std::string distribute = "auto";
  Json json() const;
};

class DistSpmv : public std::enable_shared_from_this<DistSpmv> {
public:
  /// `ctrl`: the control plane of the ranks (needed for SpmvArgs::distribute "root")
  explicit DistSpmv(SpmvArgs a, Ctrl *ctrl = nullptr);
  ~DistSpmv();
  const SpmvArgs &args() const { return a_; }
  int64_t local_rows() const { return r1_ - r0_; }
  int64_t local_nnz() const { return local_.nnz(); }
  int64_t remote_nnz() const { return remote_.nnz(); }
  int64_t remote_cols() const { return int64_t(remoteCols_.size()); }
  int64_t send_elems() const { return int64_t(sendIdx_.size()); }
  int num_peers() const;

  void setup(Ctrl *ctrl);
  bool ready() const { return dLocalRow_.get() != nullptr; }
  void add_to_graph(Graph &g);
  std::shared_ptr<const Graph> op_graph(); // the compound op's inner graph

  /// max |y - y_ref| / max(1,|y_ref|) over local rows after a run
  double check(void *stream = nullptr);
  void reset_y(void *stream = nullptr);

  // op bodies
  void scatter(void *stream) const;
  void exchange(void *stream) const;
  /// `lanes` value selecting the rocSPARSE variant of the local product
  static constexpr int kLibrary = -2;
  /// local block product into the partial y_l (or straight into y when `into_y`)
  void spmv_local(int lanes, void *stream, bool into_y = false) const;
  /// the local product as a kernel job (y_l, or y itself with `into_y`), for kernels that run
  /// it inside another launch (kern::box_move_spmv)
  kern::SpmvJob local_job(int lanes, bool into_y) const;
  /// remote block product into the partial y_r (or y += ... when `accumulate`); no launch
  /// when the remote block is empty
  void spmv_remote(void *stream, bool accumulate = false) const;
  void add(void *stream) const;
  // ipc transport
  /// credit wait, then one launch that gathers my x entries straight into every peer's remote-x
  /// buffer and signals their arrival counters
  void put(void *stream) const;
  /// wait until every peer's put of this iteration arrived in my remote-x buffer
  void wait_puts(void *stream) const;
  /// return the senders' credits (their next put may overwrite my remote-x buffer)
  void release(void *stream) const;
  bool uses_rccl() const { return useRccl_; }
  /// RCCL exchanges may be captured into hipGraphs (their preflight verified the process's
  /// capture mode); otherwise candidates with them run eagerly
  bool rccl_graph_ok() const { return rcclGraphOk_; }
  /// how the RCCL exchange is compiled into hipGraphs, or why it is not ("" = no RCCL)
  std::string rccl_capture_note() const { return rcclCaptureNote_; }
  bool uses_ipc() const { return useIpc_ && ipcReady_; }
  /// "rccl", "ipc", "rccl+ipc" (search chooses) or "none" (one rank)
  std::string transport() const;
  /// number of arrival/credit waits that timed out (0 = healthy); resets the flag
  int ipc_errors();

private:
  SpmvArgs a_;
  int64_t r0_ = 0, r1_ = 0;
  CsrHost local_, remote_;
  std::vector<int64_t> remoteCols_;          // global col of each remote x entry
  std::vector<int32_t> recvCount_, recvOff_; // per peer, into x_remote
  std::vector<int32_t> sendCount_, sendOff_; // per peer, into send buffer
  std::vector<int32_t> sendIdx_;             // local x index of each send entry
  std::vector<float> xLocal_;
  std::vector<double> yRef_;
  int lanes_ = 8;
  DeviceBuffer dLocalRow_, dLocalCol_, dLocalVal_, dRemoteRow_, dRemoteCol_, dRemoteVal_;
  DeviceBuffer dX_, dXr_, dSendIdx_, dSend_, dYl_, dYr_, dY_;
  std::shared_ptr<RcclComm> comm_;
  std::shared_ptr<RocsparseCsr> rsYl_, rsY_; // library SpMV into y_l / into y
  std::shared_ptr<Graph> form_graph_ipc(bool accumulate, const std::string &prefix);
  std::string setup_ipc(Ctrl *ctrl);
  void ipc_preflight(Ctrl *ctrl);
  /// one verified RCCL exchange under a bounded wait; "" on success, else why not
  std::string rccl_preflight_local();
  /// the random band matrix or the Matrix Market file (a_.m / nnz / bw / nnz_actual updated)
  CsrHost build_matrix();
  /// the RCCL exchange compiled into hipGraphs as the runtime compiles candidates, in the
  /// process's capture mode (or, if no workload has settled it yet, whole-schedule capture
  /// first, then child capture): collective; sets rcclGraphOk_ / rcclCaptureNote_
  void rccl_graph_preflight(Ctrl &ctrl);
  bool useRccl_ = false, useIpc_ = false, ipcReady_ = false;
  bool rcclGraphOk_ = true;
  std::string rcclCaptureNote_;
  void *flags_ = nullptr; // [arrivals from rank q | credits from rank q] (uncached, exported)
  DeviceBuffer expected_, sent_, done_, err_;
  std::vector<void *> peerXr_, peerFlags_, opened_;
  std::vector<int32_t> peerRecvOff_; // where my segment starts in peer q's remote-x buffer
  double ipcTimeoutS_ = 10.0;
  std::shared_ptr<const Graph> inner_;
  std::shared_ptr<Graph> form_graph(bool accum, const std::string &p);
  OpPtr local_op(bool accum, const std::string &p);
};

/// Horizontal fusion (fused_ops.cpp): the halo's self moves `dirs` and the SpMV's local product
/// (into y with `into_y`, else y_l) in ONE kernel launch (kern::box_move_spmv); `lanes`: the ILP
/// SpMV kernel, kern::kSpmvIlp + 1, 2 or 4 lanes per row
std::shared_ptr<GpuOp> make_move_spmv_op(std::shared_ptr<const HaloExchange> h, std::vector<int> dirs,
                                         std::shared_ptr<const DistSpmv> s, std::string name, int lanes,
                                         bool into_y);

} // namespace tz
