#include "hip_runtime.hpp"

#include "core/health.hpp"
#include "core/solve.hpp"
#include "core/util.hpp"
#include "kernels/kernels.hpp"
#include "rccl_comm.hpp"

#include <hip/hip_ext.h>
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace tz {

void hip_check(int err, const char *what, const char *file, int line) {
  if (err != hipSuccess) {
    std::ostringstream ss;
    ss << file << ":" << line << ": " << what << " failed: " << hipGetErrorString(hipError_t(err))
       << " (" << err << ")";
    throw Error(ss.str());
  }
}

void enable_roctx(bool on) {
  TraceHooks &h = trace_hooks();
  if (on) {
    h.push = [](const char *n) { roctxRangePushA(n); };
    h.pop = [] { roctxRangePop(); };
  } else {
    h.push = nullptr;
    h.pop = nullptr;
  }
}

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static hipStream_t S(void *p) { return static_cast<hipStream_t>(p); }
static hipEvent_t E(void *p) { return static_cast<hipEvent_t>(p); }

HipRuntime::HipRuntime(const HipRuntimeOpts &opts)
    : mode_(opts.mode), unroll_(std::max(1, opts.graph_unroll)), spinSync_(opts.spin_sync),
      watchdogS_(opts.watchdog_s), watchdogK_(opts.watchdog_k) {
  // TZ_TRACE: comma-separated "roctx" (the core's trace ranges to roctx) and / or "ops" (name
  // every op on stderr as eager mode issues it: hang diagnosis)
  if (const char *v = std::getenv("TZ_TRACE")) {
    const std::string t = std::string(",") + v + ",";
    if (t.find(",roctx,") != std::string::npos) enable_roctx(true);
    if (t.find(",ops,") != std::string::npos) traceOps_ = true;
  }
  TZ_CHECK(opts.n_streams >= 1, "need at least one stream");
  if (opts.device >= 0) TZ_HIP(hipSetDevice(opts.device));
  TZ_HIP(hipGetDevice(&device_));
  int nCU = 0;
  if (opts.cu_partition) {
    hipDeviceProp_t prop;
    TZ_HIP(hipGetDeviceProperties(&prop, device_));
    nCU = prop.multiProcessorCount;
  }
  for (int i = 0; i < opts.n_streams; ++i) {
    hipStream_t s = nullptr;
    if (opts.cu_partition && nCU > 0) {
      // CU ids are dealt round-robin over XCDs; give stream i every n-th CU so each stream keeps
      // a share of every XCD (and of every XCD's L2)
      std::vector<uint32_t> mask((nCU + 31) / 32, 0u);
      for (int cu = i; cu < nCU; cu += opts.n_streams) mask[cu / 32] |= 1u << (cu % 32);
      TZ_HIP(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
    } else if (i < int(opts.priorities.size())) {
      TZ_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, opts.priorities[i]));
    } else {
      TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    streams_.push_back(s);
  }
  // spare streams (never used) up to pad_streams in all: HIP deals its hardware queues to
  // streams round-robin, and hipGraph launches run their parallel branches on streams of HIP's
  // own; with 3 schedule streams one of those landed on the launch stream's queue (three
  // independent 200 us kernels: 447 us per launch; with 4-8 streams owned: 241-244 us; a host
  // node then a kernel beside two kernels: 319 -> 241 us). 6: the RCCL probe between two
  // loopback ranks also stays at its unpadded time (profiles/archive/r4_pad/)
  pad_ = opts.pad_streams >= 0 ? opts.pad_streams : tz::pad_streams();
  for (int i = opts.n_streams; i < pad_; ++i) {
    hipStream_t s = nullptr;
    TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    spare_.push_back(s);
  }
  // the device abort flag (polled by every spinning kernel) is allocated now: not inside a timed
  // run, and never inside a stream capture, where host allocations are not allowed
  kern::abort_flag();
  if (watchdogS_ > 0) {
    watchdog_ = std::thread([this] {
      // past the deadline: claim the run (one CAS on deadline_: the run's own exchange at its
      // end and this claim cannot both succeed, so a run that finishes at its deadline is either
      // aborted or not, never half), set the device abort flag (spinning kernels give up) and
      // abort the RCCL communicators (their kernels return), so the run ends and throws, and the
      // benchmarker turns that into a collectively skipped candidate; if the run still has not
      // returned after a grace period, nothing can unblock it: exit
      double grace = 0;
      uint64_t firedRun = 0;
      while (!stop_.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (grace > 0) {
          // a claimed wait: still not returned, or draining after its abort
          if (!(deadline_.abort_pending() && runGen_.load() == firedRun)) {
            grace = 0;
          } else {
            if (wtime() > grace)
              // the run is stuck where no abort reaches (e.g. a graph node that never
              // completes): leave, printing the run deadline's partial report
              exit_with_report(3, "watchdog: a hung run did not return after the abort");
            continue;
          }
        }
        if (!deadline_.try_claim(wtime())) continue; // not armed, not expired, or just ended
        firedRun = runGen_.load();
        // counted before anything can end the run, so the run waits for the abort below
        std::shared_ptr<std::atomic<int>> pending = abortsPending_;
        ++*pending;
        ++fired_;
        note_abort();
        kern::set_abort(true);
        std::fprintf(stderr,
                     "[tz] watchdog: a run exceeded its %.1f s budget (floor %.1f s + %.0f x "
                     "expected %.3g s/iter); aborting the device waits and the RCCL "
                     "communicators\n",
                     budget_.load(), watchdogS_, watchdogK_, expected_.load());
        std::fflush(stderr);
        // the abort runs on a thread of its own: it may block for seconds (it frees device
        // memory, which waits for the device), and this loop must keep watching meanwhile
        std::thread([pending] {
          if (rccl_abort_all() > 0)
            mark_domain_dead("rccl", "the watchdog aborted the RCCL communicators of a hung run");
          --*pending;
        }).detach();
        grace = wtime() + std::max(10.0, watchdogS_);
      }
    });
  }
}

double HipRuntime::watchdog_budget(int64_t n) const {
  return watchdogS_ + watchdogK_ * expected_ * double(std::max<int64_t>(1, n));
}

HipRuntime::~HipRuntime() {
  stop_ = true;
  if (watchdog_.joinable()) watchdog_.join();
  destroy_graph();
  for (void *e : events_) (void)hipEventDestroy(E(e));
  for (void *e : internal_) (void)hipEventDestroy(E(e));
  for (void *e : timerEv_)
    if (e) (void)hipEventDestroy(E(e));
  for (void *s : streams_) (void)hipStreamDestroy(S(s));
  for (void *s : spare_) (void)hipStreamDestroy(S(s));
}

std::string HipRuntime::device_name() const {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device_) != hipSuccess) return "?";
  return std::string(prop.name) + " (" + prop.gcnArchName + ")";
}

void *HipRuntime::event(int e) {
  TZ_CHECK(e >= 0, "negative event id");
  while (int(events_.size()) <= e) {
    hipEvent_t ev;
    TZ_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    events_.push_back(ev);
  }
  return events_[e];
}

void *HipRuntime::internal_event() {
  if (internalUsed_ == internal_.size()) {
    hipEvent_t ev;
    TZ_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    internal_.push_back(ev);
  }
  return internal_[internalUsed_++];
}

void *HipRuntime::native_stream(int stream) {
  TZ_CHECK(stream >= 0 && stream < num_streams(), "stream " << stream << " out of range");
  return streams_[stream];
}

int HipRuntime::stream_index(const void *native) const {
  // an op being captured on the origin stream answers for its own logical stream
  if (captureAs_ >= 0 && native == streams_[0]) return captureAs_;
  for (size_t i = 0; i < streams_.size(); ++i)
    if (streams_[i] == native) return int(i);
  return -1;
}

void HipRuntime::launch(const GpuOp &op, int stream) { op.launch(native_stream(stream), *this); }

void HipRuntime::event_record(int e, int stream) {
  TZ_HIP(hipEventRecord(E(event(e)), S(native_stream(stream))));
}

void HipRuntime::stream_wait_event(int stream, int e) {
  TZ_HIP(hipStreamWaitEvent(S(native_stream(stream)), E(event(e)), 0));
}

void HipRuntime::event_sync(int e) {
  hipEvent_t ev = E(event(e));
  if (spinSync_) {
    // busy-poll: the host wakes as soon as the event completes (no blocking-wait latency)
    hipError_t r;
    while ((r = hipEventQuery(ev)) == hipErrorNotReady) {
    }
    TZ_HIP(r);
  } else {
    TZ_HIP(hipEventSynchronize(ev));
  }
}

void HipRuntime::stream_sync(int stream) {
  hipStream_t s = S(native_stream(stream));
  if (spinSync_) {
    hipError_t r;
    while ((r = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    TZ_HIP(r);
  } else {
    TZ_HIP(hipStreamSynchronize(s));
  }
}

void HipRuntime::stream_wait(int waiter, int waitee) {
  hipEvent_t ev = E(internal_event());
  TZ_HIP(hipEventRecord(ev, S(native_stream(waitee))));
  TZ_HIP(hipStreamWaitEvent(S(native_stream(waiter)), ev, 0));
}

void HipRuntime::device_sync() {
  // bounded like a run: work still in flight after a run returned (RCCL's own streams, copy
  // engines) must not block the caller forever where no watchdog looks
  guarded(watchdogS_, "a device synchronization", [] { TZ_HIP(hipDeviceSynchronize()); });
}

void HipRuntime::destroy_exec(void *exec) {
  if (!exec) return;
  (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec));
  auto it = graphOf_.find(exec);
  if (it != graphOf_.end()) {
    (void)hipGraphDestroy(static_cast<hipGraph_t>(it->second));
    graphOf_.erase(it);
  }
}

void HipRuntime::destroy_graph() {
  if (graphExecR_) { // always owned here, never by a slot
    destroy_exec(graphExecR_);
    graphExecR_ = nullptr;
    remR_ = 0;
  }
  if (!slots_.empty()) {
    // the current graphs are borrowed from a slot
    for (Slot &s : slots_) {
      destroy_exec(s.exec);
      destroy_exec(s.execU);
    }
    slots_.clear();
    graphExec_ = graphExecU_ = nullptr;
    graphNodes_ = graphEdges_ = 0;
    return;
  }
  if (graphExec_) {
    destroy_exec(graphExec_);
    graphExec_ = nullptr;
    graphNodes_ = graphEdges_ = 0;
  }
  if (graphExecU_) {
    destroy_exec(graphExecU_);
    graphExecU_ = nullptr;
  }
}

std::map<std::string, int> HipRuntime::graph_node_types() const {
  std::map<std::string, int> out;
  if (!graphExec_) return out;
  auto it = graphOf_.find(graphExec_);
  if (it == graphOf_.end()) return out;
  hipGraph_t g = static_cast<hipGraph_t>(it->second);
  size_t n = 0;
  TZ_HIP(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) TZ_HIP(hipGraphGetNodes(g, nodes.data(), &n));
  for (hipGraphNode_t x : nodes) {
    hipGraphNodeType t;
    TZ_HIP(hipGraphNodeGetType(x, &t));
    const char *name = "other";
    switch (t) {
    case hipGraphNodeTypeKernel: name = "kernel"; break;
    case hipGraphNodeTypeMemcpy: name = "memcpy"; break;
    case hipGraphNodeTypeMemset: name = "memset"; break;
    case hipGraphNodeTypeHost: name = "host"; break;
    case hipGraphNodeTypeGraph: name = "child_graph"; break;
    case hipGraphNodeTypeEmpty: name = "empty"; break;
    case hipGraphNodeTypeWaitEvent: name = "event_wait"; break;
    case hipGraphNodeTypeEventRecord: name = "event_record"; break;
    default: break;
    }
    ++out[name];
  }
  return out;
}

bool HipRuntime::recordable(const Sequence &seq) const {
  for (const auto &e : seq.entries) {
    const OpClass c = e.op->op_class();
    if (c == OpClass::Cpu) {
      // only host no-ops can be dropped from a replay
      if (e.op->kind() != "NoOp" || e.op->cost_us() > 0) return false;
    } else if (c == OpClass::BoundGpu) {
      if (!static_cast<const BoundGpuOp &>(*e.op).unbound()->capturable()) return false;
    }
  }
  return true;
}

void HipRuntime::set_mode(ExecMode m) {
  if (m != mode_) {
    destroy_graph();
    mode_ = m;
  }
}

void *HipRuntime::build_graph(int iterations, size_t &nodesOut, size_t &edgesOut) {
  const int nS = num_streams();
  SyncModel model(nS);
  // per stream, in issue order: the graph nodes that stand for each issued GPU op. An op that
  // enqueued nothing stands for its own dependencies (no empty node: every empty node costs a
  // barrier packet — ~10 us — at replay), an op that enqueued a fan-out for all its tails.
  using NodeSet = std::vector<void *>;
  std::vector<std::vector<NodeSet>> nodes(nS);
  size_t edges = 0;
  hipGraph_t graph = nullptr;
  // a schedule with RCCL ops between ranks is built the way the RCCL preflight found exact
  bool rccl = false;
  for (const auto &e : seq_.entries)
    if (e.op->op_class() == OpClass::BoundGpu &&
        static_cast<const BoundGpuOp &>(*e.op).unbound()->order_domain() == "rccl")
      rccl = true;
  const CaptureMode mode = rccl && rccl_multi_rank() ? rccl_capture_mode() : capture_mode();
  {
    GraphBuilder gb(streams_, mode);
    // replaying the sequence `iterations` times through one model orders iteration i+1 after
    // iteration i exactly as the schedule's closing host syncs do in eager mode
    for (int it = 0; it < iterations; ++it)
      for (const auto &e : seq_.entries) {
        const BoundOp &op = *e.op;
        if (op.op_class() == OpClass::BoundGpu) {
          const auto &b = static_cast<const BoundGpuOp &>(op);
          const int s = b.stream();
          TZ_CHECK(s >= 0 && s < nS, "stream " << s << " out of range");
          // dependencies: previous op on this stream + the latest op of every other stream that
          // the schedule's events / host syncs make complete before this one is issued
          NodeSet deps;
          if (!nodes[s].empty()) deps = nodes[s].back();
          for (int t = 0; t < nS; ++t) {
            if (t == s) continue;
            const int k = model.known(s, t);
            if (k > 0) {
              const NodeSet &d = nodes[t][size_t(k) - 1];
              deps.insert(deps.end(), d.begin(), d.end());
            }
          }
          std::sort(deps.begin(), deps.end());
          deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
          // captured on the origin stream: the op still sees its own logical stream index
          // (communicator choice, per-stream resources) through stream_index()
          captureAs_ = s;
          NodeSet tails;
          try {
            tails = gb.add(s, deps, [&](void *cs) { b.unbound()->launch(cs, *this); });
          } catch (...) {
            captureAs_ = -1;
            throw;
          }
          captureAs_ = -1;
          if (tails.empty()) {
            nodes[s].push_back(deps); // enqueued nothing: stands for its dependencies
          } else {
            nodes[s].push_back(tails);
            edges += deps.size();
          }
        }
        model.apply(op);
      }
    graph = static_cast<hipGraph_t>(gb.finish());
  }
  try {
    size_t real = 0;
    TZ_HIP(hipGraphGetNodes(graph, nullptr, &real)); // the capture has ended: safe to inspect
    hipGraphExec_t exec = nullptr;
    TZ_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    graphOf_[exec] = graph; // destroyed with the exec (destroy_exec)
    graph = nullptr;
    nodesOut = real;
    edgesOut = edges;
    TZ_LOG(Debug, "graph mode (" << capture_mode_name(mode) << " capture): " << iterations
                                 << " iteration(s), " << real << " nodes, " << edges << " edges");
    // upload once so the first timed launch does not pay for it
    try {
      TZ_HIP(hipGraphUpload(exec, S(streams_[0])));
      TZ_HIP(hipStreamSynchronize(S(streams_[0])));
    } catch (...) {
      destroy_exec(exec);
      throw;
    }
    return exec;
  } catch (...) {
    if (graph) (void)hipGraphDestroy(graph);
    throw;
  }
}

namespace {
std::atomic<int> g_capture{int(CaptureMode::Schedule)};
std::atomic<bool> g_captureForced{false};
std::atomic<int> g_rcclCapture{int(CaptureMode::Schedule)};
std::atomic<int> g_padStreams{6};
} // namespace

CaptureMode capture_mode() { return CaptureMode(g_capture.load()); }

bool capture_mode_forced() { return g_captureForced.load(); }

void set_graph_capture(const std::string &how) {
  TZ_CHECK(how == "schedule" || how == "child" || how == "auto",
           "graph capture must be schedule, child or auto (got " << how << ")");
  g_capture = int(how == "child" ? CaptureMode::Child : CaptureMode::Schedule);
  g_captureForced = how != "auto";
}

CaptureMode rccl_capture_mode() {
  return capture_mode_forced() ? capture_mode() : CaptureMode(g_rcclCapture.load());
}

std::atomic<bool> g_rcclCaptureSettled{false};
void set_rccl_capture_mode(CaptureMode m) {
  g_rcclCapture = int(m);
  g_rcclCaptureSettled = true;
}
bool rccl_capture_settled() { return g_rcclCaptureSettled.load(); }

const char *capture_mode_name(CaptureMode m) {
  return m == CaptureMode::Child ? "child" : "schedule";
}

GraphBuilder::GraphBuilder(const std::vector<void *> &streams, CaptureMode mode)
    : streams_(streams), mode_(mode) {
  TZ_CHECK(!streams_.empty(), "a graph build needs at least one stream");
  if (mode_ == CaptureMode::Child) {
    hipGraph_t g = nullptr;
    TZ_HIP(hipGraphCreate(&g, 0));
    graph_ = g;
    return;
  }
  hipStream_t origin = S(streams_[0]);
  TZ_LOG(Debug, "capture: begin");
  TZ_HIP(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
  capturing_ = true;
}

int pad_streams() { return g_padStreams.load(); }

void set_default_pad_streams(int n) {
  TZ_CHECK(n >= 0 && n <= 64, "pad streams must be in [0, 64] (got " << n << ")");
  g_padStreams = n;
}

GraphBuilder::~GraphBuilder() { abandon(); }

void GraphBuilder::abandon() {
  if (capturing_) {
    capturing_ = false;
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(S(streams_[0]), &g);
    if (g) (void)hipGraphDestroy(g);
  }
  if (graph_) {
    (void)hipGraphDestroy(static_cast<hipGraph_t>(graph_));
    graph_ = nullptr;
  }
}

std::vector<void *> GraphBuilder::add(int stream, const std::vector<void *> &depsP,
                                      const std::function<void(void *)> &launch) {
  TZ_CHECK(stream >= 0 && stream < int(streams_.size()), "stream " << stream << " out of range");
  std::vector<hipGraphNode_t> deps;
  for (void *d : depsP) deps.push_back(static_cast<hipGraphNode_t>(d));
  std::vector<void *> tails;
  if (mode_ == CaptureMode::Child) {
    hipStream_t st = S(streams_[stream]);
    hipGraph_t captured = nullptr;
    TZ_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    try {
      launch(st);
    } catch (...) {
      (void)hipStreamEndCapture(st, &captured);
      if (captured) (void)hipGraphDestroy(captured);
      throw;
    }
    TZ_HIP(hipStreamEndCapture(st, &captured));
    size_t nsub = 0;
    const hipError_t rn = hipGraphGetNodes(captured, nullptr, &nsub); // its capture has ended
    if (rn == hipSuccess && nsub > 0) {
      hipGraphNode_t node = nullptr;
      const hipError_t r = hipGraphAddChildGraphNode(&node, static_cast<hipGraph_t>(graph_),
                                                     deps.data(), deps.size(), captured);
      (void)hipGraphDestroy(captured); // the child node holds its own copy
      TZ_HIP(r);
      tails.push_back(node);
    } else {
      (void)hipGraphDestroy(captured);
      TZ_HIP(rn);
    }
    return tails;
  }
  TZ_CHECK(capturing_, "graph build already finished");
  // every op is enqueued on the origin stream, behind exactly its schedule dependencies
  // (whatever was captured before): in a graph only the edges exist, not the streams, so one
  // capture stream suffices. It also keeps every side stream an op forks internally (RCCL's
  // own streams, copy engines) joined to the origin itself: HIP 7.0's hipStreamEndCapture
  // recursed without end when RCCL's streams had joined the capture through other forked
  // streams (profiles/archive/r4_capture/self_torchrt2.log)
  hipStream_t origin = S(streams_[0]);
  TZ_LOG(Debug, "capture: op of stream " << stream << " behind " << deps.size() << " node(s)");
  TZ_HIP(hipStreamUpdateCaptureDependencies(origin, deps.empty() ? nullptr : deps.data(), deps.size(),
                                            hipStreamSetCaptureDependencies));
  launch(origin);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const hipGraphNode_t *d = nullptr;
  size_t nd = 0;
  TZ_HIP(hipStreamGetCaptureInfo_v2(origin, &cs, nullptr, nullptr, &d, &nd));
  TZ_CHECK(cs == hipStreamCaptureStatusActive, "stream capture was invalidated by an op's launch");
  std::vector<hipGraphNode_t> after(d, d + nd);
  std::sort(after.begin(), after.end());
  std::vector<hipGraphNode_t> before = deps;
  std::sort(before.begin(), before.end());
  if (after == before) return tails; // enqueued nothing
  for (hipGraphNode_t n : after) tails.push_back(n);
  return tails;
}

void *GraphBuilder::finish() {
  if (mode_ == CaptureMode::Child) {
    void *g = graph_;
    graph_ = nullptr;
    return g;
  }
  TZ_CHECK(capturing_, "graph build already finished");
  capturing_ = false;
  hipGraph_t g = nullptr;
  TZ_LOG(Debug, "capture: ending");
  TZ_HIP(hipStreamEndCapture(S(streams_[0]), &g));
  TZ_CHECK(g != nullptr, "stream capture produced no graph");
  TZ_LOG(Debug, "capture: ended");
  return g;
}

void HipRuntime::set_graph_unroll(int u) {
  u = std::max(1, u);
  if (u != unroll_) {
    destroy_graph();
    unroll_ = u;
  }
}

void HipRuntime::prepare(const Sequence &seq) {
  destroy_graph();
  seq_ = seq;
  internalUsed_ = 0;
  expected_ = 0; // a new schedule: the watchdog floor alone bounds its first run
  event(std::max(0, seq.num_events() - 1)); // provision the event pool
  if (mode_ == ExecMode::Graph && recordable(seq)) {
    size_t n = 0, e = 0;
    graphExec_ = build_graph(1, graphNodes_, graphEdges_);
    if (unroll_ > 1) graphExecU_ = build_graph(unroll_, n, e);
  }
}

void HipRuntime::prepare_many(const std::vector<Sequence> &seqs) {
  destroy_graph();
  std::vector<Slot> slots;
  try {
    for (const Sequence &s : seqs) {
      prepare(s); // compiles into graphExec_ / graphExecU_ (owned here until moved)
      Slot sl;
      sl.seq = s;
      sl.exec = graphExec_;
      sl.execU = graphExecU_;
      sl.nodes = graphNodes_;
      sl.edges = graphEdges_;
      graphExec_ = graphExecU_ = nullptr;
      slots.push_back(std::move(sl));
    }
  } catch (...) {
    for (Slot &s : slots) {
      destroy_exec(s.exec);
      destroy_exec(s.execU);
    }
    throw;
  }
  slots_ = std::move(slots);
  int events = 1;
  for (const Slot &s : slots_) events = std::max(events, s.seq.num_events());
  event(events - 1);
  if (!slots_.empty()) select(0);
}

void HipRuntime::select(size_t k) {
  TZ_CHECK(k < slots_.size(), "slot " << k << " out of range (" << slots_.size() << ")");
  if (graphExecR_ && k != slot_) { // the remainder graph belongs to the previous slot's schedule
    destroy_exec(graphExecR_);
    graphExecR_ = nullptr;
    remR_ = 0;
  }
  const Slot &s = slots_[k];
  seq_ = s.seq;
  graphExec_ = s.exec;
  graphExecU_ = s.execU;
  graphNodes_ = s.nodes;
  graphEdges_ = s.edges;
  internalUsed_ = 0;
  slot_ = k;
  expected_ = s.expected;
}

double HipRuntime::run_device_timed(int64_t n) {
  for (void *&e : timerEv_)
    if (!e) {
      hipEvent_t ev;
      TZ_HIP(hipEventCreate(&ev));
      e = ev;
    }
  TZ_HIP(hipEventRecord(E(timerEv_[0]), S(streams_[0])));
  run(n);
  TZ_HIP(hipEventRecord(E(timerEv_[1]), S(streams_[0])));
  TZ_HIP(hipEventSynchronize(E(timerEv_[1])));
  float ms = 0;
  TZ_HIP(hipEventElapsedTime(&ms, E(timerEv_[0]), E(timerEv_[1])));
  return double(ms) * 1e-3;
}

std::vector<HipRuntime::Span> HipRuntime::trace(const Sequence &seq, int iterations) {
  TZ_CHECK(iterations >= 1, "iterations must be positive");
  const Sequence keep = seq_;
  seq_ = seq;
  event(std::max(0, seq.num_events() - 1));
  std::vector<hipEvent_t> evs;
  auto timing_event = [&] {
    hipEvent_t e;
    TZ_HIP(hipEventCreate(&e));
    evs.push_back(e);
    return e;
  };
  struct Pending {
    size_t span;
    hipEvent_t a, b;
  };
  std::vector<Span> spans;
  std::vector<Pending> pending;
  std::string err;
  try {
    TZ_HIP(hipDeviceSynchronize());
    hipEvent_t base = timing_event();
    TZ_HIP(hipEventRecord(base, S(streams_[0])));
    TZ_HIP(hipEventSynchronize(base));
    const double h0 = wtime();
    for (int it = 0; it < iterations; ++it) {
      internalUsed_ = 0;
      for (const auto &e : seq.entries) {
        const BoundOp &op = *e.op;
        if (op.op_class() == OpClass::BoundGpu) {
          const int st = static_cast<const BoundGpuOp &>(op).stream();
          hipEvent_t a = timing_event(), b = timing_event();
          TZ_HIP(hipEventRecord(a, S(native_stream(st))));
          op.run(*this);
          TZ_HIP(hipEventRecord(b, S(native_stream(st))));
          pending.push_back({spans.size(), a, b});
          spans.push_back({op.name(), st, it, 0, 0});
        } else {
          const double t0 = wtime();
          op.run(*this);
          spans.push_back({op.name(), -1, it, (t0 - h0) * 1e6, (wtime() - h0) * 1e6});
        }
      }
    }
    TZ_HIP(hipDeviceSynchronize());
    for (const Pending &p : pending) {
      float ta = 0, tb = 0;
      TZ_HIP(hipEventElapsedTime(&ta, base, p.a));
      TZ_HIP(hipEventElapsedTime(&tb, base, p.b));
      spans[p.span].start_us = double(ta) * 1e3;
      spans[p.span].end_us = double(tb) * 1e3;
    }
  } catch (const std::exception &e) {
    err = e.what();
  }
  for (hipEvent_t e : evs) (void)hipEventDestroy(e);
  seq_ = keep;
  internalUsed_ = 0;
  if (!err.empty()) throw Error(err);
  return spans;
}

Json chrome_trace(const std::vector<HipRuntime::Span> &spans) {
  Json ev = Json::array();
  int maxStream = -1;
  for (const auto &s : spans) maxStream = std::max(maxStream, s.stream);
  auto meta = [&](int tid, const std::string &name) {
    Json m, a;
    m["name"] = "thread_name";
    m["ph"] = "M";
    m["pid"] = int64_t(0);
    m["tid"] = int64_t(tid);
    a["name"] = name;
    m["args"] = a;
    ev.push_back(m);
  };
  meta(0, "host");
  for (int s = 0; s <= maxStream; ++s) meta(s + 1, "stream " + std::to_string(s));
  for (const auto &s : spans) {
    Json j, a;
    j["name"] = s.name;
    j["ph"] = "X";
    j["pid"] = int64_t(0);
    j["tid"] = int64_t(s.stream + 1);
    j["ts"] = s.start_us;
    j["dur"] = std::max(0.0, s.end_us - s.start_us);
    a["iteration"] = int64_t(s.iteration);
    j["args"] = a;
    ev.push_back(j);
  }
  Json out;
  out["traceEvents"] = ev;
  out["displayTimeUnit"] = "ns";
  return out;
}

void HipRuntime::guarded(double budget, const char *what, const std::function<void()> &body) {
  if (guarding_) { // nested (an op of a run synchronizes the device): the run's deadline covers it
    body();
    return;
  }
  struct Flag {
    bool &f;
    explicit Flag(bool &x) : f(x) { f = true; }
    ~Flag() { f = false; }
  } flag(guarding_);
  ++runGen_;
  // a device abort flag still set (an earlier abort whose drain was cut short, or a transport
  // preflight that left it): drain and clear it, or every spinning kernel of this run would
  // give up at once
  if (kern::abort_set()) {
    (void)hipDeviceSynchronize();
    kern::set_abort(false);
  }
  if (watchdogS_ > 0) {
    budget_ = budget;
    deadline_.arm(wtime() + budget);
  }
  // the end of the guarded wait: one exchange against the watchdog's claim
  auto finish = [&] {
    if (!deadline_.finish()) return;
    // aborted: let every kernel the abort released drain before the flag is cleared for the
    // next run (draining keeps the watchdog's grace exit armed: a drain that never ends hits it)
    (void)hipDeviceSynchronize();
    kern::set_abort(false);
    // the communicator abort normally ends well before the run returns; give it a bounded wait
    // so that the caller sees RCCL marked dead (and the domain agreement sees it) on return
    for (const double until = wtime() + 10.0; abortsPending_->load() > 0 && wtime() < until;)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    deadline_.drained();
    TZ_THROW("watchdog: " << what << " exceeded its " << budget_.load() << " s budget and was aborted");
  };
  try {
    body();
  } catch (...) {
    finish(); // throws the watchdog's error instead when it had claimed the wait
    throw;
  }
  finish();
}

void HipRuntime::run(int64_t n) {
  const double t0 = wtime();
  guarded(watchdog_budget(n), "the run", [&] { run_impl(n); });
  // what the next run of this schedule may take: its longest per-iteration time so far
  const double per = (wtime() - t0) / double(std::max<int64_t>(1, n));
  expected_ = std::max(expected_.load(), per);
  if (!slots_.empty() && slot_ < slots_.size()) slots_[slot_].expected = expected_;
}

void HipRuntime::precompile(int64_t n) {
  if (!graphExec_ || !graphExecU_ || unroll_ <= 1) return;
  const int64_t r = n % unroll_;
  if (r <= 1 || (graphExecR_ && remR_ == r)) return;
  if (graphExecR_) {
    destroy_exec(graphExecR_);
    graphExecR_ = nullptr;
    remR_ = 0;
  }
  size_t nodes = 0, edges = 0;
  graphExecR_ = build_graph(int(r), nodes, edges);
  remR_ = r;
}

void HipRuntime::run_impl(int64_t n) {
  if (graphExec_) {
    hipStream_t origin = S(streams_[0]);
    int64_t i = 0;
    if (graphExecU_)
      for (; i + unroll_ <= n; i += unroll_)
        TZ_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graphExecU_), origin));
    if (graphExecR_ && n - i == remR_) {
      TZ_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graphExecR_), origin));
      i = n;
    }
    for (; i < n; ++i) TZ_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graphExec_), origin));
    stream_sync(0);
  } else {
    const bool traced = trace_hooks().push != nullptr;
    for (int64_t i = 0; i < n; ++i) {
      internalUsed_ = 0;
      for (const auto &e : seq_.entries) {
        if (traceOps_) std::fprintf(stderr, "[tz] op %s\n", e.op->name().c_str());
        if (traced) {
          TraceRange r(e.op->name().c_str());
          e.op->run(*this);
        } else {
          e.op->run(*this);
        }
      }
    }
  }
}

} // namespace tz
