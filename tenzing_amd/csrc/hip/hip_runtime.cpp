#include "hip_runtime.hpp"

#include "core/util.hpp"

#include <hip/hip_ext.h>
#include <hip/hip_runtime_api.h>

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

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static hipStream_t S(void *p) { return static_cast<hipStream_t>(p); }
static hipEvent_t E(void *p) { return static_cast<hipEvent_t>(p); }

HipRuntime::HipRuntime(const HipRuntimeOpts &opts) : mode_(opts.mode), watchdogS_(opts.watchdog_s) {
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
  if (watchdogS_ > 0) {
    watchdog_ = std::thread([this] {
      while (!stop_.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
        const double d = deadline_.load();
        if (d > 0 && wtime() > d) {
          std::fprintf(stderr,
                       "[tz] watchdog: schedule iteration exceeded %.1f s (deadlocked "
                       "communication?); aborting\n",
                       watchdogS_);
          std::fflush(stderr);
          std::_Exit(3);
        }
      }
    });
  }
}

HipRuntime::~HipRuntime() {
  stop_ = true;
  if (watchdog_.joinable()) watchdog_.join();
  destroy_graph();
  for (void *e : events_) hipEventDestroy(E(e));
  for (void *e : internal_) hipEventDestroy(E(e));
  for (void *s : streams_) hipStreamDestroy(S(s));
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

void HipRuntime::capture_guard(int stream) {
  if (!capturing_) return;
  auto &ap = applied_[stream];
  for (size_t k = 0; k < hostSynced_.size(); ++k) {
    if (ap.size() <= k) ap.resize(hostSynced_.size(), 0);
    if (!ap[k]) {
      ap[k] = 1;
      wait(stream, event(hostSynced_[k]));
    }
  }
}

// During capture, HIP (ROCm 7.2) crashes in hipStreamEndCapture when a stream waits on an event
// it recorded itself; such waits (and repeated waits on the same recording) are redundant by
// stream order, so they are dropped while capturing.
void HipRuntime::record(void *ev, int stream) {
  TZ_HIP(hipEventRecord(E(ev), S(native_stream(stream))));
  if (capturing_) {
    capRec_[ev] = stream;
    for (auto it = capWaited_.begin(); it != capWaited_.end();)
      it = it->second == ev ? capWaited_.erase(it) : std::next(it);
  }
}

void HipRuntime::wait(int stream, void *ev) {
  if (capturing_) {
    auto it = capRec_.find(ev);
    if (it == capRec_.end() || it->second == stream) return;
    if (!capWaited_.insert({stream, ev}).second) return;
  }
  TZ_HIP(hipStreamWaitEvent(S(native_stream(stream)), E(ev), 0));
}

void HipRuntime::launch(const GpuOp &op, int stream) {
  capture_guard(stream);
  op.launch(native_stream(stream), *this);
}

void HipRuntime::event_record(int e, int stream) {
  capture_guard(stream);
  record(event(e), stream);
}

void HipRuntime::stream_wait_event(int stream, int e) {
  capture_guard(stream);
  wait(stream, event(e));
}

void HipRuntime::event_sync(int e) {
  if (capturing_) {
    hostSynced_.push_back(e);
    return;
  }
  TZ_HIP(hipEventSynchronize(E(event(e))));
}

void HipRuntime::stream_sync(int stream) {
  if (capturing_) {
    // host waits for the stream: represent as an internal event the later enqueues depend on
    const int e = int(events_.size());
    record(event(e), stream);
    hostSynced_.push_back(e);
    return;
  }
  TZ_HIP(hipStreamSynchronize(S(native_stream(stream))));
}

void HipRuntime::stream_wait(int waiter, int waitee) {
  capture_guard(waiter);
  capture_guard(waitee);
  void *ev = internal_event();
  record(ev, waitee);
  wait(waiter, ev);
}

void HipRuntime::device_sync() { TZ_HIP(hipDeviceSynchronize()); }

void HipRuntime::destroy_graph() {
  if (graphExec_) {
    hipGraphExecDestroy(static_cast<hipGraphExec_t>(graphExec_));
    graphExec_ = nullptr;
    graphNodes_ = 0;
  }
}

bool HipRuntime::capturable(const Sequence &seq) const {
  for (const auto &e : seq.entries) {
    const OpClass c = e.op->op_class();
    if (c == OpClass::Cpu) {
      // only host no-ops can be captured
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

void HipRuntime::prepare(const Sequence &seq) {
  destroy_graph();
  seq_ = seq;
  internalUsed_ = 0;
  event(std::max(0, seq.num_events() - 1)); // provision the event pool
  if (mode_ != ExecMode::Graph || !capturable(seq)) return;

  // record the whole schedule into one hipGraph by capturing stream 0 and forking the others
  hipStream_t origin = S(streams_[0]);
  TZ_HIP(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
  capturing_ = true;
  hostSynced_.clear();
  applied_.assign(streams_.size(), {});
  capRec_.clear();
  capWaited_.clear();
  try {
    void *fork = internal_event();
    record(fork, 0);
    for (size_t i = 1; i < streams_.size(); ++i) wait(int(i), fork);
    for (const auto &e : seq_.entries) {
      TZ_LOG(Debug, "capture: " << e.op->desc());
      e.op->run(*this);
    }
    // join every stream into the origin (host syncs at the end need no extra edges: the join
    // already orders all work before the graph's completion)
    for (size_t i = 1; i < streams_.size(); ++i) {
      void *join = internal_event();
      record(join, int(i));
      wait(0, join);
    }
  } catch (...) {
    capturing_ = false;
    hipGraph_t g = nullptr;
    hipStreamEndCapture(origin, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  capturing_ = false;
  hipGraph_t graph = nullptr;
  TZ_LOG(Debug, "capture: end capture");
  TZ_HIP(hipStreamEndCapture(origin, &graph));
  TZ_LOG(Debug, "capture: ended");
  size_t n = 0;
  if (std::getenv("TZ_GRAPH_COUNT_NODES")) TZ_HIP(hipGraphGetNodes(graph, nullptr, &n));
  TZ_LOG(Debug, "capture: " << n << " nodes; instantiating");
  hipGraphExec_t exec = nullptr;
  TZ_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  TZ_LOG(Debug, "capture: instantiated");
  TZ_HIP(hipGraphDestroy(graph));
  graphExec_ = exec;
  graphNodes_ = n;
  // upload once so the first timed launch does not pay for it
  TZ_HIP(hipGraphUpload(exec, origin));
  TZ_HIP(hipStreamSynchronize(origin));
}

void HipRuntime::run_eager_once() {
  for (const auto &e : seq_.entries) e.op->run(*this);
}

void HipRuntime::run(int64_t n) {
  if (watchdogS_ > 0) deadline_ = wtime() + watchdogS_ * double(std::max<int64_t>(1, n));
  if (graphExec_) {
    hipStream_t origin = S(streams_[0]);
    for (int64_t i = 0; i < n; ++i)
      TZ_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graphExec_), origin));
    TZ_HIP(hipStreamSynchronize(origin));
  } else {
    for (int64_t i = 0; i < n; ++i) {
      internalUsed_ = 0;
      run_eager_once();
    }
  }
  deadline_ = 0;
}

} // namespace tz
