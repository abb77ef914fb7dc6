// All-pairs link probe: what every ordered pair of ranks moves through one IPC mapping, by the
// halo's kernel put and by the SDMA engines, with every rank sending at once.
//
// Round s (1 <= s < P) is a permutation: rank r writes into rank (r + s) % P's buffer while it
// receives from (r - s) % P, so each round loads P distinct directed links together, as an
// exchange does. On an 8-GPU node the 7 rounds cover all 56 directed xGMI links; on loopback
// ranks (one GPU) every "link" is the same HBM. The halo link probe measures only the links its
// faces use; this one shows the whole fabric, e.g. whether every pair is one hop.
//
// Reference: none (the reference relies on CUDA-aware MPI and never measures its fabric).
#include "workloads.hpp"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "core/util.hpp"
#include "hip/hip_runtime.hpp"

#include <hip/hip_runtime_api.h>

namespace tz {

namespace {
// wait for `e` for at most `limit_s` (polling; hipEventSynchronize has no bound): false if it did
// not complete in time. TZ_FAIL_TRANSPORTS containing "link_matrix_stall" (tests) treats every
// wait as one that never completes.
bool wait_event_bounded(hipEvent_t e, double limit_s) {
  const char *f = std::getenv("TZ_FAIL_TRANSPORTS");
  const bool stall = f && (std::string(",") + f + ",").find(",link_matrix_stall,") != std::string::npos;
  const double end = wtime() + limit_s;
  for (;;) {
    const hipError_t q = stall ? hipErrorNotReady : hipEventQuery(e);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) TZ_HIP(q);
    if (wtime() > end) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}
} // namespace

LinkMatrix link_matrix(Ctrl &ctrl, size_t bytes, int iters, double wait_limit_s) {
  TZ_CHECK(wait_limit_s > 0, "wait_limit_s must be positive");
  const int P = ctrl.size(), R = ctrl.rank();
  TZ_CHECK(iters >= 1, "iters must be positive");
  constexpr size_t kRow = 4096; // elements per row of the put's box (32 KiB)
  TZ_CHECK(bytes >= kRow * 8 && bytes % (kRow * 8) == 0 && bytes / (kRow * 8) < (size_t(1) << 31),
           "bytes must be a positive multiple of " << kRow * 8);
  LinkMatrix out;
  out.bytes = double(bytes);
  out.iters = iters;
  out.put.assign(size_t(P), std::vector<double>(size_t(P), -1.0));
  out.sdma = out.put;
  if (P < 2) {
    out.why = "one rank: no pairs";
    return out;
  }
  const size_t H = sizeof(hipIpcMemHandle_t);
  // Every rank makes the same control-plane calls whatever fails locally; failures are agreed.
  std::string err, mine;
  DeviceBuffer src, dst, done, flag;
  try {
    src = DeviceBuffer(bytes);
    TZ_HIP(hipMemset(src.get(), 0x3f, bytes));
    dst = DeviceBuffer(bytes, /*peerWritten=*/true);
    done = DeviceBuffer(kern::kMaxBoxes * sizeof(unsigned int));
    TZ_HIP(hipMemset(done.get(), 0, done.bytes()));
    flag = DeviceBuffer(sizeof(unsigned long long));
    TZ_HIP(hipMemset(flag.get(), 0, flag.bytes()));
    TZ_HIP(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    std::memset(&h, 0, sizeof(h));
    TZ_HIP(hipIpcGetMemHandle(&h, dst.get()));
    mine = node_identity() + std::string(reinterpret_cast<const char *>(&h), H);
  } catch (const std::exception &e) {
    err = std::string("export: ") + e.what();
    mine.clear();
  }
  const std::vector<std::string> all = ctrl.allgather(mine);
  std::vector<void *> peer(size_t(P), nullptr);
  auto close_all = [&] {
    for (void *&p : peer)
      if (p) {
        (void)hipIpcCloseMemHandle(p);
        p = nullptr;
      }
  };
  if (err.empty()) {
    try {
      const std::string me = node_identity();
      for (int q = 0; q < P; ++q) {
        if (q == R) continue;
        const std::string &blob = all[size_t(q)];
        TZ_CHECK(blob.size() == kNodeIdBytes + H, "rank " << q << " exported no handle");
        TZ_CHECK(blob.compare(0, kNodeIdBytes, me) == 0, "rank " << q << " runs on another node");
        hipIpcMemHandle_t h;
        std::memcpy(&h, blob.data() + kNodeIdBytes, H);
        TZ_HIP(hipIpcOpenMemHandle(&peer[size_t(q)], h, hipIpcMemLazyEnablePeerAccess));
      }
    } catch (const std::exception &e) {
      err = std::string("map: ") + e.what();
    }
  }
  double bad = err.empty() ? 0.0 : 1.0;
  ctrl.allreduce_max(&bad, 1);
  if (bad != 0.0) {
    close_all();
    ctrl.barrier();
    out.why = err.empty() ? "failed on another rank" : err;
    return out;
  }
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<double> row(size_t(2 * P), -1.0); // [put to q | sdma to q]
  try {
    TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    TZ_HIP(hipEventCreate(&e0));
    TZ_HIP(hipEventCreate(&e1));
  } catch (const std::exception &e) {
    err = std::string("probe: ") + e.what();
  }
  // the same barriers on every rank whatever fails locally: a rank that failed only skips its
  // transfers. Every device wait is bounded: a transfer that has not completed in time (a link
  // that stalls) fails this rank's probe, and its buffers, mappings and stream are then left as
  // they are (releasing them would wait for the stuck transfer) -- the caller gets a result
  // that says why instead of a hang
  bool stuck = false;
  for (int kind = 0; kind < 2; ++kind) {
    for (int shift = 1; shift < P; ++shift) {
      const int q = (R + shift) % P;
      ctrl.barrier();
      if (!err.empty()) continue;
      try {
        TZ_HIP(hipEventRecord(e0, s));
        for (int it = 0; it < iters; ++it) {
          if (kind == 0) {
            // the halo's put kernel (signalling launch at the default put width); the arrival
            // counter is a local one, nobody waits for it
            kern::MoveDesc m;
            m.src = src.as<double>();
            m.dst = static_cast<double *>(peer[size_t(q)]);
            m.len = int32_t(kRow);
            m.n1 = int32_t(bytes / (kRow * 8));
            m.n2 = m.n3 = 1;
            m.s1 = int64_t(kRow);
            m.s2 = m.s3 = 0;
            kern::MoveSignal sig;
            sig.done = done.as<unsigned int>();
            sig.flag[0] = flag.as<unsigned long long>();
            kern::box_move_many_signal(&m, 1, sig, s);
          } else {
            TZ_HIP(hipMemcpyAsync(peer[size_t(q)], src.get(), bytes, hipMemcpyDeviceToDeviceNoCU, s));
          }
        }
        TZ_HIP(hipEventRecord(e1, s));
        if (!wait_event_bounded(e1, wait_limit_s)) {
          stuck = true;
          err = "probe: " + std::string(kind == 0 ? "kernel put" : "SDMA copy") + " to rank " +
                std::to_string(q) + " did not complete within " + std::to_string(wait_limit_s) + " s";
          continue;
        }
        float ms = 0;
        TZ_HIP(hipEventElapsedTime(&ms, e0, e1));
        row[size_t(kind * P + q)] = ms > 0 ? double(bytes) * iters / (double(ms) * 1e-3) / 1e9 : -1.0;
      } catch (const std::exception &e) {
        err = std::string("probe: ") + e.what();
      }
    }
  }
  // every rank has stopped writing into its peers before any buffer is unmapped or freed
  if (s && !stuck) (void)hipStreamSynchronize(s);
  double anyStuck = stuck ? 1.0 : 0.0;
  ctrl.allreduce_max(&anyStuck, 1);
  out.stuck = anyStuck != 0.0;
  if (out.stuck) {
    // a transfer somewhere has not completed: it may still write into any rank's buffer, so
    // nothing is unmapped, freed or destroyed (a process exit reclaims it)
    src.leak();
    dst.leak();
    done.leak();
    flag.leak();
  } else {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    close_all();
  }
  std::string enc(reinterpret_cast<const char *>(row.data()), row.size() * sizeof(double));
  const std::vector<std::string> rows = ctrl.allgather(err.empty() ? enc : std::string());
  for (int r = 0; r < P; ++r) {
    const std::string &x = rows[size_t(r)];
    if (x.size() != row.size() * sizeof(double)) continue;
    std::vector<double> v(row.size());
    std::memcpy(v.data(), x.data(), x.size());
    for (int q = 0; q < P; ++q) {
      out.put[size_t(r)][size_t(q)] = v[size_t(q)];
      out.sdma[size_t(r)][size_t(q)] = v[size_t(P + q)];
    }
  }
  double failed = err.empty() ? 0.0 : 1.0;
  ctrl.allreduce_max(&failed, 1);
  if (failed != 0.0) out.why = err.empty() ? "probe failed on another rank" : err;
  return out;
}

} // namespace tz
