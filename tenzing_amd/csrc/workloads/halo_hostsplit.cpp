// Halo workload, host split: a share of every face through node shared host memory over each
// GPU's own PCIe link, beside the xGMI IPC put (halo_relay.cpp has the face split).
#include "halo_internal.hpp"

namespace tz {

// ---------------------------------------------------------------- host split (PCIe beside xGMI)
//
// Per iteration, for every face direction i (share f of its box by host memory, in chunks c):
//   sender r:    split_put_direct  share A -> receiver R's device receive buffer (IPC), slot i
//                hs_put_host       wait my inbox credit i (lag 1); per chunk c: pack it into R's
//                                  inbox region of ghost side -d_i (kernel stores over r's PCIe
//                                  link), then store ++count into R's inbox arrival (c, i)
//   receiver R:  hs_wait           device arrivals of every direction
//                hs_unpack         unpack the device shares, device credits (IPC); per chunk c:
//                                  wait inbox arrival (c, i), DMA the chunk from the inbox into
//                                  the receive buffer behind A; inbox credits (store ++count
//                                  into r's inbox credit i); unpack the chunks
// With several chunks the receiver's DMA of chunk c can overlap the sender's stores of chunk
// c + 1 (a PCIe link carries 68 GB/s both ways at once vs 55 / 39 one way, profiles/archive/r3_pcie);
// measured, the per-chunk hand-offs cost more than that wins (profiles/archive/r3_hs_chunks), so the
// default is one chunk: all stores, then one DMA.
// Every host-memory counter has exactly one writer, so plain release stores publish them (no
// PCIe AtomicOps). Same induction as IPC puts: puts wait only for credits of the previous
// iteration, so no schedule can deadlock.

std::string HaloExchange::setup_hostsplit(Ctrl *ctrl) {
  // Collective whatever fails locally: one bcast, two allreduce agreements, one barrier.
  const int nd = ndirs();
  std::string err;
  std::string token = ctrl->rank() == 0 ? std::to_string(uint64_t(wtime() * 1e6) ^ (uint64_t(::getpid()) << 20)) : "";
  ctrl->bcast(token, 0);
  auto name_of = [&](int r) { return "/tz_hs_" + token + "_" + std::to_string(r); };
  // layout, the same on every rank: the counters, then one region per ghost side of a face
  const std::vector<int> faces = relay_faces();
  hsRegion_.assign(size_t(nd), 0);
  size_t at = round_up(int64_t(size_t(hsChunks_ + 1) * nd * 8), 4096);
  for (int i : faces) {
    const int o = opp_[i];
    size_t most = 0;
    for (double f : a_.hostsplit_fracs) {
      kern::BoxDesc A, B, u = make_box(a_, dirs_[o], true, xoff_, sy_, sz_, sq_);
      u.buf = nullptr;
      split_box(u, f, A, B);
      size_t sum = 0;
      for (const kern::BoxDesc &c : chunk_box(B, hs_parts(f)))
        sum += size_t(round_up(int64_t(c.len) * c.n1 * c.n2 * c.n3, 16)) * sizeof(double);
      most = std::max(most, sum);
    }
    hsRegion_[size_t(o)] = at;
    at += size_t(round_up(int64_t(most), 4096));
  }
  const size_t bytes = at;
  try {
    hsMine_ = SharedHostBuffer::create(name_of(ctrl->rank()), bytes);
    hsBook_ = DeviceBuffer(size_t(2 * hsChunks_ + 2) * size_t(nd) * 8);
    TZ_HIP(hipMemset(hsBook_.get(), 0, hsBook_.bytes()));
    TZ_HIP(hipDeviceSynchronize());
  } catch (const std::exception &e) {
    err = std::string("create: ") + e.what();
  }
  double bad = err.empty() ? 0.0 : 1.0;
  ctrl->allreduce_max(&bad, 1); // every inbox exists (or nobody maps any)
  if (bad == 0) {
    try {
      hsPeer_.resize(size_t(a_.size));
      for (int i : faces)
        for (int q : {nbr_[i], nbr_[opp_[i]]})
          if (q != a_.rank && !hsPeer_[size_t(q)].host())
            hsPeer_[size_t(q)] = SharedHostBuffer::open(name_of(q), bytes);
    } catch (const std::exception &e) {
      err = std::string("map: ") + e.what();
    }
  }
  double bad2 = err.empty() ? 0.0 : 1.0;
  ctrl->allreduce_max(&bad2, 1); // every peer mapped what it needs: the names can go
  hsMine_.unlink();
  if (bad != 0 || bad2 != 0) {
    hsPeer_.clear();
    hsMine_ = SharedHostBuffer();
    return err.empty() ? "failed on another rank" : err;
  }
  TZ_LOG(Info, "host split: " << bytes / 1048576.0 << " MiB inbox per rank in shared host memory");
  return "";
}

int HaloExchange::hs_parts(double frac) const {
  // the same number of chunks for every face: a chunk launch then holds all faces or none, so a
  // face's arrival counter (MoveSignal::count, by position in the launch) keeps its position
  // whichever share the schedule uses; sender and receiver see the same box shapes
  int parts = hsChunks_;
  for (int i : relay_faces()) {
    kern::BoxDesc A, B, b = make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_);
    b.buf = nullptr;
    split_box(b, frac, A, B);
    parts = std::min(parts, int(chunk_box(B, hsChunks_).size()));
  }
  return std::max(parts, 1);
}

void HaloExchange::hs_put_host(const std::vector<int> &faces, double frac, void *stream) const {
  TZ_CHECK(ready() && hsReady_, "host split not set up");
  TZ_CHECK(!faces.empty() && faces.size() <= size_t(kern::kMaxBoxes), "bad host-split face group");
  const int nd = ndirs(), C = hsChunks_;
  unsigned long long *book = hsBook_.as<unsigned long long>();
  // my previous shares have been consumed: their credits in my inbox (slots C nd + i)
  kern::ipc_wait(static_cast<const unsigned long long *>(hsMine_.dev()) + size_t(C) * nd,
                 book + size_t(C) * nd, faces.data(), int(faces.size()), err_.as<int>(),
                 ipcTimeoutS_, stream, /*lag=*/1);
  std::vector<std::vector<kern::BoxDesc>> chunks;
  for (int i : faces) {
    const SharedHostBuffer &peer = hsPeer_[size_t(nbr_[i])];
    TZ_CHECK(peer.dev(), "rank " << nbr_[i] << "'s inbox is not mapped");
    kern::BoxDesc A, B;
    split_box(make_box(a_, dirs_[i], false, xoff_, sy_, sz_, sq_), frac, A, B);
    B.buf = reinterpret_cast<double *>(static_cast<char *>(peer.dev()) + hsRegion_[size_t(opp_[i])]);
    chunks.push_back(chunk_box(B, hs_parts(frac)));
  }
  // one launch per chunk index, in order: chunk c is complete (and flagged) while c + 1 is
  // still crossing the link
  for (int c = 0; c < C; ++c) {
    std::vector<kern::BoxDesc> bs;
    kern::MoveSignal sig;
    sig.done = done_.as<unsigned int>() + size_t(3 * nd + faces.front()) * kern::kMaxBoxes;
    sig.count = book + size_t(C + 1 + c) * nd; // one per face, in `faces` order
    for (size_t k = 0; k < faces.size(); ++k) {
      if (size_t(c) >= chunks[k].size()) continue;
      const int i = faces[k];
      sig.flag[bs.size()] = static_cast<unsigned long long *>(hsPeer_[size_t(nbr_[i])].dev()) +
                            size_t(c) * nd + i;
      sig.store_mask |= 1ull << bs.size();
      bs.push_back(chunks[k][size_t(c)]);
    }
    if (!bs.empty()) kern::box_pack_many_signal(grid(), bs.data(), int(bs.size()), sig, stream);
  }
}

void HaloExchange::hs_wait(const std::vector<int> &dirs, const std::vector<int> &faces,
                           void *stream) const {
  TZ_CHECK(ready() && hsReady_, "host split not set up");
  (void)faces; // the host chunks are waited for in hs_unpack, one at a time
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_), expected_.as<unsigned long long>(),
                 dirs.data(), int(dirs.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/0);
}

void HaloExchange::hs_unpack(const std::vector<int> &dirs, const std::vector<int> &faces,
                             double frac, void *stream) const {
  TZ_CHECK(ready() && hsReady_, "host split not set up");
  const int nd = ndirs(), C = hsChunks_;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the device shares first: unpacked, their buffers' credits returned
  std::vector<kern::BoxDesc> bs;
  std::vector<std::vector<kern::BoxDesc>> chunks; // per face of `faces` in `dirs`
  std::vector<int> split;                         // those faces
  for (int i : dirs) {
    check_pipelined(i);
    const kern::BoxDesc u = unpack_box(opp_[i]); // buf = my receive buffer of ghost side -d_i
    if (std::find(faces.begin(), faces.end(), i) == faces.end()) {
      bs.push_back(u);
      continue;
    }
    kern::BoxDesc A, B;
    split_box(u, frac, A, B); // B.buf: behind A in the receive buffer
    bs.push_back(A);
    split.push_back(i);
    chunks.push_back(chunk_box(B, hs_parts(frac)));
  }
  for (size_t k = 0; k < bs.size(); k += kern::kMaxBoxes)
    kern::box_copy_many(grid(), bs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, bs.size() - k)),
                        true, stream);
  const std::vector<unsigned long long *> credits = credit_ptrs(dirs);
  kern::ipc_signal(credits.data(), int(credits.size()), stream);
  if (split.empty()) return;
  // the host shares chunk by chunk: each DMA (the copy engine reads host memory coherently) as
  // soon as its chunk arrived, while the sender stores the next
  const unsigned long long *inbox = static_cast<const unsigned long long *>(hsMine_.dev());
  unsigned long long *book = hsBook_.as<unsigned long long>();
  std::vector<kern::BoxDesc> hbs;
  for (int c = 0; c < C; ++c) {
    std::vector<int> here;
    for (size_t k = 0; k < split.size(); ++k)
      if (size_t(c) < chunks[k].size()) here.push_back(split[k]);
    if (here.empty()) break;
    kern::ipc_wait(inbox + size_t(c) * nd, book + size_t(c) * nd, here.data(), int(here.size()),
                   err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/0);
    for (size_t k = 0; k < split.size(); ++k) {
      if (size_t(c) >= chunks[k].size()) continue;
      const kern::BoxDesc &x = chunks[k][size_t(c)];
      const size_t off = size_t(x.buf - chunks[k][0].buf) * sizeof(double);
      const size_t bytes = size_t(x.len) * x.n1 * x.n2 * x.n3 * sizeof(double);
      TZ_HIP(hipMemcpyAsync(x.buf, static_cast<const char *>(hsMine_.host()) + hsRegion_[size_t(opp_[split[k]])] + off,
                            bytes, hipMemcpyHostToDevice, s));
      hbs.push_back(x);
    }
  }
  // the inbox regions are free again (the DMAs are done, stream order): the senders' credits,
  // one counter per face, in `faces` order
  std::vector<unsigned long long *> hostCredits;
  for (int i : faces) {
    const SharedHostBuffer &peer = hsPeer_[size_t(nbr_[opp_[i]])];
    TZ_CHECK(peer.dev(), "rank " << nbr_[opp_[i]] << "'s inbox is not mapped");
    hostCredits.push_back(static_cast<unsigned long long *>(peer.dev()) + size_t(C) * nd + i);
  }
  kern::ipc_signal(hostCredits.data(), int(hostCredits.size()), stream,
                   book + size_t(2 * C + 1) * nd);
  for (size_t k = 0; k < hbs.size(); k += kern::kMaxBoxes)
    kern::box_copy_many(grid(), hbs.data() + k, int(std::min<size_t>(kern::kMaxBoxes, hbs.size() - k)),
                        true, stream);
}

void HaloExchange::hostsplit_preflight(Ctrl *ctrl) {
  // one verified exchange per offered share before the search may use it; a failure turns it
  // off on every rank (the other transports remain)
  std::vector<int> local, remote;
  for (int i = 0; i < ndirs(); ++i) {
    if (direct_[i]) local.push_back(i);
    else if (ipc_[i]) remote.push_back(i);
  }
  const std::vector<int> faces = relay_faces();
  double bad = 0;
  std::string why;
  const double keep = ipcTimeoutS_;
  ipcTimeoutS_ = std::min(ipcTimeoutS_, preflight_wait_s());
  int gen = 0;
  for (double f : a_.hostsplit_fracs) {
    // a new generation of values per share: data left in a buffer or cache by the previous
    // exchange fails the check instead of passing as current
    init_grid(nullptr, 1 + gen++ % 3);
    TZ_HIP(hipDeviceSynchronize());
    ctrl->barrier();
    if (bad == 0) {
      try {
        if (!local.empty()) direct_group(local, nullptr);
        split_put_direct(remote, f, nullptr);
        hs_put_host(faces, f, nullptr);
        hs_wait(remote, faces, nullptr);
        hs_unpack(remote, faces, f, nullptr);
        TZ_HIP(hipDeviceSynchronize());
      } catch (const std::exception &ex) {
        bad = 1;
        why = std::string("host split preflight: ") + ex.what();
      }
    }
    ctrl->barrier();
    if (bad == 0) {
      try {
        const int e = ipc_errors();
        const uint64_t cells = check_grid();
        if (e || cells) {
          bad = 1;
          why = "host split preflight (share " + std::to_string(f) + "): " + std::to_string(e) +
                " wait timeout(s), " + std::to_string(cells) + " wrong cells";
        }
      } catch (const std::exception &ex) {
        bad = 1;
        why = std::string("host split preflight check: ") + ex.what();
      }
    }
    ctrl->allreduce_max(&bad, 1);
    if (bad != 0) break;
  }
  ipcTimeoutS_ = keep;
  if (bad != 0) {
    hsReady_ = false;
    hsWhy_ = why.empty() ? "preflight failed on another rank" : why;
    TZ_LOG(Warn, "host split disabled: " << hsWhy_);
    reset_ipc_counters(ctrl);
    TZ_CHECK(a_.hostsplit != "force", "host split forced but " << hsWhy_);
  }
  init_grid();
}

std::vector<kern::BoxDesc> HaloExchange::chunk_box(const kern::BoxDesc &b, int parts) {
  int32_t n[3] = {b.n1, b.n2, b.n3};
  const int64_t st[3] = {b.s1, b.s2, b.s3};
  int k = 2;
  for (int j = 1; j >= 0; --j)
    if (n[j] > n[k]) k = j;
  parts = std::max(1, std::min(parts, n[k]));
  std::vector<kern::BoxDesc> out;
  int64_t off = 0;
  int32_t at = 0;
  for (int c = 0; c < parts; ++c) {
    kern::BoxDesc x = b;
    int32_t *nx[3] = {&x.n1, &x.n2, &x.n3};
    *nx[k] = n[k] / parts + (c < n[k] % parts ? 1 : 0);
    x.grid_off = b.grid_off + int64_t(at) * st[k];
    x.buf = b.buf ? b.buf + off : nullptr;
    at += *nx[k];
    off += round_up(int64_t(x.len) * x.n1 * x.n2 * x.n3, 16);
    out.push_back(x);
  }
  return out;
}

} // namespace tz
