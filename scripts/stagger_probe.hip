// When does each branch of a multi-stream schedule start on the device?
//
// k single-workgroup kernels, one per stream, each stamps wall_clock64 at its start and end.
// Launch forms: eager launches on k streams; one hipGraph captured with fork/join events (the
// way the runtime compiles a schedule); k one-kernel graphs launched on k streams. Prints one
// JSON line per (form, k, kernel length): each kernel's start offset from the earliest start, in
// us, median over the timed launches, and the wall time per launch.
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/stagger_probe scripts/stagger_probe.hip
//   /tmp/stagger_probe [iters]
//
// Then the back-to-back form (unrolled graphs, no host sync between copies); see below.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      std::exit(1);                                                                               \
    }                                                                                             \
  } while (0)

__global__ void stamp_k(long long ticks, long long *out, int slot) {
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(1);
    t = wall_clock64();
  }
  if (threadIdx.x == 0) {
    out[2 * slot] = t0;
    out[2 * slot + 1] = t;
  }
}

__global__ void empty_join_k() {}

__global__ void stamp_seq_k(long long ticks, long long *out, unsigned *counter) {
  // as stamp_k, the slot taken in completion order (a graph replays fixed arguments)
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(1);
    t = wall_clock64();
  }
  if (threadIdx.x == 0) {
    const unsigned slot = atomicAdd(counter, 1u);
    out[2 * slot] = t0;
    out[2 * slot + 1] = t;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Probe {
  int k;
  long long ticks;
  double tick_us;
  std::vector<hipStream_t> s;
  long long *d = nullptr;
  std::vector<long long> h;

  void launch_eager() {
    for (int i = 0; i < k; ++i) hipLaunchKernelGGL(stamp_k, 1, 64, 0, s[i], ticks, d, i);
  }
  // start offsets (us) of the last launch, relative to the earliest
  std::vector<double> offsets() {
    CK(hipMemcpy(h.data(), d, sizeof(long long) * 2 * k, hipMemcpyDeviceToHost));
    long long t0 = h[0];
    for (int i = 0; i < k; ++i) t0 = std::min(t0, h[2 * i]);
    std::vector<double> o(k);
    for (int i = 0; i < k; ++i) o[i] = double(h[2 * i] - t0) * tick_us;
    return o;
  }
};

static void report(const char *form, Probe &p, double us, std::vector<std::vector<double>> &offs,
                   double wall) {
  std::printf("{\"form\": \"%s\", \"k\": %d, \"kernel_us\": %.0f, \"start_offset_us\": [", form,
              p.k, us);
  for (int i = 0; i < p.k; ++i) {
    std::vector<double> v;
    for (auto &o : offs) v.push_back(o[i]);
    std::sort(v.begin(), v.end());
    std::printf("%s%.1f", i ? ", " : "", v[v.size() / 2]);
  }
  std::printf("], \"wall_us_per_launch\": %.1f}\n", wall);
  std::fflush(stdout);
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20;
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const double tick_us = 1000.0 / rate_khz;
  std::vector<hipStream_t> streams(4);
  for (auto &st : streams) CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  long long *d;
  CK(hipMalloc(&d, sizeof(long long) * 16));

  for (double us : {5.0, 50.0, 200.0}) {
    for (int k : {1, 2, 3, 4}) {
      Probe p{k, (long long)(us / tick_us), tick_us, streams, d, std::vector<long long>(2 * k)};
      p.s.resize(k);
      std::vector<std::vector<double>> offs;

      // eager
      p.launch_eager();
      CK(hipDeviceSynchronize());
      double t0 = now_us();
      for (int it = 0; it < iters; ++it) {
        p.launch_eager();
        CK(hipDeviceSynchronize());
        offs.push_back(p.offsets());
      }
      report("eager", p, us, offs, (now_us() - t0) / iters);

      // one graph, fork/join events (whole-schedule capture)
      std::vector<hipEvent_t> ev(2 * k);
      for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      hipGraph_t g;
      CK(hipStreamBeginCapture(p.s[0], hipStreamCaptureModeThreadLocal));
      CK(hipEventRecord(ev[0], p.s[0]));
      for (int i = 1; i < k; ++i) CK(hipStreamWaitEvent(p.s[i], ev[0], 0));
      p.launch_eager();
      for (int i = 1; i < k; ++i) {
        CK(hipEventRecord(ev[k + i], p.s[i]));
        CK(hipStreamWaitEvent(p.s[0], ev[k + i], 0));
      }
      CK(hipStreamEndCapture(p.s[0], &g));
      hipGraphExec_t ge;
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, p.s[0]));
      CK(hipDeviceSynchronize());
      offs.clear();
      t0 = now_us();
      for (int it = 0; it < iters; ++it) {
        CK(hipGraphLaunch(ge, p.s[0]));
        CK(hipDeviceSynchronize());
        offs.push_back(p.offsets());
      }
      report("graph", p, us, offs, (now_us() - t0) / iters);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));

      // k one-kernel graphs, one per stream
      std::vector<hipGraphExec_t> ges(k);
      for (int i = 0; i < k; ++i) {
        hipGraph_t gi;
        CK(hipStreamBeginCapture(p.s[i], hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(stamp_k, 1, 64, 0, p.s[i], p.ticks, d, i);
        CK(hipStreamEndCapture(p.s[i], &gi));
        CK(hipGraphInstantiate(&ges[i], gi, nullptr, nullptr, 0));
        CK(hipGraphDestroy(gi));
      }
      for (int i = 0; i < k; ++i) CK(hipGraphLaunch(ges[i], p.s[i]));
      CK(hipDeviceSynchronize());
      offs.clear();
      t0 = now_us();
      for (int it = 0; it < iters; ++it) {
        for (int i = 0; i < k; ++i) CK(hipGraphLaunch(ges[i], p.s[i]));
        CK(hipDeviceSynchronize());
        offs.push_back(p.offsets());
      }
      report("graph_per_stream", p, us, offs, (now_us() - t0) / iters);
      for (auto ge2 : ges) CK(hipGraphExecDestroy(ge2));
      for (auto &e : ev) CK(hipEventDestroy(e));
    }
  }

  // Back to back, as the bench times a schedule: U copies of the fork/join pattern (or of k
  // kernels in a row on one stream) captured into one graph, R launches, no host sync between.
  // Per copy: device span (earliest start to latest end) and the gap to the next copy's start.
  const int U = 10, R = 5;
  long long *du;
  CK(hipMalloc(&du, sizeof(long long) * 2 * 4 * U));
  std::vector<long long> hu(2 * 4 * U);
  std::vector<hipEvent_t> ev(2 * 4 * U);
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (double us : {5.0, 20.0, 50.0}) {
    const long long ticks = (long long)(us / tick_us);
    for (int serial = 0; serial < 4; ++serial) {
      for (int k : {1, 2, 3, 4}) {
        if (serial == 1 && k == 1) continue;
        hipGraph_t g;
        hipStream_t s0 = streams[0];
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
        std::vector<hipGraphNode_t> prev; // form 2: the previous copy's kernels
        for (int u = 0; u < U; ++u) {
          if (serial == 3) {
            // a join kernel: one empty kernel behind all of the previous copy's kernels, the
            // next copy's kernels behind it alone (k deps once instead of k x k)
            if (!prev.empty()) {
              CK(hipStreamUpdateCaptureDependencies(s0, prev.data(), prev.size(),
                                                    hipStreamSetCaptureDependencies));
              hipLaunchKernelGGL(empty_join_k, 1, 64, 0, s0);
              hipStreamCaptureStatus cs;
              const hipGraphNode_t *d = nullptr;
              size_t nd = 0;
              CK(hipStreamGetCaptureInfo_v2(s0, &cs, nullptr, nullptr, &d, &nd));
              prev.assign(d, d + nd);
            }
            std::vector<hipGraphNode_t> cur;
            for (int i = 0; i < k; ++i) {
              CK(hipStreamUpdateCaptureDependencies(s0, prev.empty() ? nullptr : prev.data(), prev.size(),
                                                    hipStreamSetCaptureDependencies));
              hipLaunchKernelGGL(stamp_k, 1, 64, 0, s0, ticks, du, u * k + i);
              hipStreamCaptureStatus cs;
              const hipGraphNode_t *d = nullptr;
              size_t nd = 0;
              CK(hipStreamGetCaptureInfo_v2(s0, &cs, nullptr, nullptr, &d, &nd));
              cur.insert(cur.end(), d, d + nd);
            }
            prev = cur;
            continue;
          }
          if (serial == 2) {
            // the runtime's form: every kernel captured on ONE stream behind exactly its
            // dependencies (all kernels of the previous copy), set with
            // hipStreamUpdateCaptureDependencies
            std::vector<hipGraphNode_t> cur;
            for (int i = 0; i < k; ++i) {
              CK(hipStreamUpdateCaptureDependencies(s0, prev.empty() ? nullptr : prev.data(), prev.size(),
                                                    hipStreamSetCaptureDependencies));
              hipLaunchKernelGGL(stamp_k, 1, 64, 0, s0, ticks, du, u * k + i);
              hipStreamCaptureStatus cs;
              const hipGraphNode_t *d = nullptr;
              size_t nd = 0;
              CK(hipStreamGetCaptureInfo_v2(s0, &cs, nullptr, nullptr, &d, &nd));
              cur.insert(cur.end(), d, d + nd);
            }
            prev = cur;
            continue;
          }
          if (serial) {
            for (int i = 0; i < k; ++i)
              hipLaunchKernelGGL(stamp_k, 1, 64, 0, s0, ticks, du, u * k + i);
            continue;
          }
          hipEvent_t *e = &ev[2 * 4 * u];
          CK(hipEventRecord(e[0], s0));
          for (int i = 1; i < k; ++i) CK(hipStreamWaitEvent(streams[i], e[0], 0));
          for (int i = 0; i < k; ++i)
            hipLaunchKernelGGL(stamp_k, 1, 64, 0, streams[i], ticks, du, u * k + i);
          for (int i = 1; i < k; ++i) {
            CK(hipEventRecord(e[4 + i], streams[i]));
            CK(hipStreamWaitEvent(s0, e[4 + i], 0));
          }
        }
        CK(hipStreamEndCapture(s0, &g));
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s0));
        CK(hipDeviceSynchronize());
        double t0 = now_us();
        for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s0));
        CK(hipDeviceSynchronize());
        const double wall = (now_us() - t0) / (R * U);
        CK(hipMemcpy(hu.data(), du, sizeof(long long) * 2 * k * U, hipMemcpyDeviceToHost));
        std::vector<double> span, gap, last_start;
        for (int u = 0; u < U; ++u) {
          long long a = hu[2 * u * k], b = hu[2 * u * k + 1], ls = a;
          for (int i = 0; i < k; ++i) {
            a = std::min(a, hu[2 * (u * k + i)]);
            ls = std::max(ls, hu[2 * (u * k + i)]);
            b = std::max(b, hu[2 * (u * k + i) + 1]);
          }
          span.push_back(double(b - a) * tick_us);
          last_start.push_back(double(ls - a) * tick_us);
          if (u + 1 < U) {
            long long n = hu[2 * (u + 1) * k];
            for (int i = 0; i < k; ++i) n = std::min(n, hu[2 * ((u + 1) * k + i)]);
            gap.push_back(double(n - b) * tick_us);
          }
        }
        auto med = [](std::vector<double> v) {
          std::sort(v.begin(), v.end());
          return v[v.size() / 2];
        };
        std::printf("{\"form\": \"%s\", \"k\": %d, \"kernel_us\": %.0f, \"us_per_copy\": %.1f, "
                    "\"span_us\": %.1f, \"last_start_us\": %.1f, \"gap_to_next_us\": %.1f}\n",
                    serial == 3 ? "unrolled_joinkernel" : serial == 2 ? "unrolled_origin" : serial ? "unrolled_serial" : "unrolled_forkjoin", k, us, wall, med(span),
                    med(last_start), med(gap));
        std::fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
    }
  }

  // Back to back, one copy per hipGraphLaunch (R launches, no host sync between): the per-launch
  // fork from and join back to the launch stream, vs the in-graph fork/join above.
  {
    const int RL = 10;
    long long *dl;
    unsigned *cnt;
    CK(hipMalloc(&dl, sizeof(long long) * 2 * 4 * RL));
    CK(hipMalloc(&cnt, sizeof(unsigned)));
    std::vector<long long> hl(2 * 4 * RL);
    for (double us : {5.0, 50.0, 200.0}) {
      const long long ticks = (long long)(us / tick_us);
      for (int k : {1, 2, 3, 4}) {
        hipGraph_t g;
        hipStream_t s0 = streams[0];
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(ev[0], s0));
        for (int i = 1; i < k; ++i) CK(hipStreamWaitEvent(streams[i], ev[0], 0));
        for (int i = 0; i < k; ++i) hipLaunchKernelGGL(stamp_seq_k, 1, 64, 0, streams[i], ticks, dl, cnt);
        for (int i = 1; i < k; ++i) {
          CK(hipEventRecord(ev[4 + i], streams[i]));
          CK(hipStreamWaitEvent(s0, ev[4 + i], 0));
        }
        CK(hipStreamEndCapture(s0, &g));
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s0));
        CK(hipDeviceSynchronize());
        CK(hipMemset(cnt, 0, sizeof(unsigned)));
        CK(hipDeviceSynchronize());
        double t0 = now_us();
        for (int r = 0; r < RL; ++r) CK(hipGraphLaunch(ge, s0));
        CK(hipDeviceSynchronize());
        const double wall = (now_us() - t0) / RL;
        CK(hipMemcpy(hl.data(), dl, sizeof(long long) * 2 * k * RL, hipMemcpyDeviceToHost));
        std::vector<std::pair<long long, long long>> v;
        for (int i = 0; i < k * RL; ++i) v.push_back({hl[2 * i], hl[2 * i + 1]});
        std::sort(v.begin(), v.end());
        std::vector<double> span, gap, last_start;
        for (int r = 0; r < RL; ++r) {
          long long a = v[r * k].first, b = 0, ls = 0;
          for (int i = 0; i < k; ++i) {
            b = std::max(b, v[r * k + i].second);
            ls = std::max(ls, v[r * k + i].first);
          }
          span.push_back(double(b - a) * tick_us);
          last_start.push_back(double(ls - a) * tick_us);
          if (r + 1 < RL) gap.push_back(double(v[(r + 1) * k].first - b) * tick_us);
        }
        auto med = [](std::vector<double> x) {
          std::sort(x.begin(), x.end());
          return x[x.size() / 2];
        };
        std::printf("{\"form\": \"launch_b2b_forkjoin\", \"k\": %d, \"kernel_us\": %.0f, "
                    "\"us_per_launch\": %.1f, \"span_us\": %.1f, \"last_start_us\": %.1f, "
                    "\"gap_to_next_us\": %.1f}\n",
                    k, us, wall, med(span), med(last_start), med(gap));
        std::fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
    }
    CK(hipFree(dl));
    CK(hipFree(cnt));
  }
  for (auto &e : ev) CK(hipEventDestroy(e));
  CK(hipFree(du));
  CK(hipFree(d));
  for (auto st : streams) CK(hipStreamDestroy(st));
  return 0;
}
