// HIP runtime: the MI355X execution platform for candidate schedules.
//
// Parity: reference Platform (include/tenzing/platform.hpp:147-219: cudaStream pool via
// make_n_streams, ResourceMap Event->cudaEvent_t, CudaEventPool :221-242), the CUDA sync ops'
// run() (src/cuda/ops_cuda.cpp:48-168) and the benchmark hot loop (src/benchmarker.cpp:93-97).
// MI355X design:
//  * N non-blocking HIP streams, optionally with priorities or disjoint CU masks
//    (hipExtStreamCreateWithCUMask: a stream can be pinned to a subset of the 256 CUs / 8 XCDs,
//    turning "which CUs" into a schedulable resource);
//  * a pool of timing-disabled hipEvents indexed by the schedule's abstract event ids;
//  * two execution modes for one schedule: Eager (host issues every op each iteration, like the
//    reference) and Graph (the schedule is compiled once into a hipGraph and replayed with one
//    hipGraphLaunch per iteration). The whole schedule is one stream capture (GraphBuilder):
//    its happens-before relation is replayed in the same vector-clock model the synchronizer
//    uses, and every GPU op is enqueued on its stream with that stream's capture dependencies
//    set to exactly the nodes the schedule's events / host syncs imply. Host synchronizations
//    therefore cost nothing inside a replay, and RCCL ops are ordinary concurrent nodes;
//  * a watchdog: a run of n iterations gets `watchdog_s + watchdog_k * expected * n` seconds,
//    where `expected` is the longest per-iteration time of an earlier run of the same prepared
//    schedule (0 before the first one: the floor alone bounds the first, short, sizing run).
//    Past the deadline it sets the device abort flag (every spinning kernel gives up) and aborts
//    the process's RCCL communicators (ncclCommAbort; the "rccl" ordering domain is marked dead,
//    health.hpp), so the blocked run returns and throws; the benchmarker turns that into a
//    candidate every rank skips. A run that still does not return after a grace period ends the
//    process with a diagnostic.
#pragma once

#include "core/benchmark.hpp"
#include "core/deadline_claim.hpp"

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace tz {

enum class ExecMode { Eager, Graph };

struct HipRuntimeOpts {
  int device = -1;             // -1: keep current device
  int n_streams = 2;
  std::vector<int> priorities; // optional per-stream priorities
  bool cu_partition = false;   // give each stream a disjoint, XCD-balanced CU mask
  ExecMode mode = ExecMode::Eager;
  double watchdog_s = 0;       // deadline floor per run, seconds (0 = no watchdog)
  double watchdog_k = 50;      // ... plus this many times the expected time of the run
  int graph_unroll = 1;        // iterations per hipGraph launch in Graph mode
  bool spin_sync = true;       // host syncs busy-poll (blocking waits measured no faster)
  int pad_streams = -1;        // streams owned at least (spares never used); -1: pad_streams()
};

// ExecutorRunner first: the Python bindings expose HipRuntime through that base
class HipRuntime : public ExecutorRunner, public Executor {
public:
  explicit HipRuntime(const HipRuntimeOpts &opts);
  ~HipRuntime() override;
  HipRuntime(const HipRuntime &) = delete;
  HipRuntime &operator=(const HipRuntime &) = delete;

  // Executor
  int num_streams() const override { return int(streams_.size()); }
  int pad_streams() const { return std::max(pad_, int(streams_.size())); }
  /// the watchdog's budget for n iterations plus its grace before the process exit (0: no
  /// watchdog, unbounded)
  double run_budget(int64_t n) const override {
    return watchdogS_ > 0 ? watchdog_budget(n) + std::max(10.0, watchdogS_) : 0.0;
  }
  void launch(const GpuOp &op, int stream) override;
  void event_record(int event, int stream) override;
  void stream_wait_event(int stream, int event) override;
  void event_sync(int event) override;
  void stream_sync(int stream) override;
  void stream_wait(int waiter, int waitee) override;
  void device_sync() override;
  void *native_stream(int stream) override;
  int stream_index(const void *native) const override;

  // ExecutorRunner
  void prepare(const Sequence &seq) override;
  void run(int64_t n) override;
  /// run(n) bracketed by timing events on stream 0 (every op of a schedule follows the first
  /// event, and the schedule's closing host syncs precede the last): device seconds
  double run_device_timed(int64_t n) override;
  int64_t batch_multiple() const override { return graphExecU_ ? unroll_ : 1; }
  /// graph mode with unroll u > 1: also compile a graph of the n % u iterations a run(n) leaves
  /// after its whole unrolled launches, so that run(n) launches ONE graph for them instead of
  /// n % u one-iteration graphs (each launch boundary of a multi-stream graph costs ~20 us;
  /// profiles/r5_branch/). Call it before a timed run(n); kept until the schedule, the unroll or
  /// the selected slot changes.
  void precompile(int64_t n);
  /// graph mode: every sequence is compiled once and kept; select() switches without rebuilding
  void prepare_many(const std::vector<Sequence> &seqs) override;
  void select(size_t k) override;

  void set_mode(ExecMode m);
  ExecMode mode() const { return mode_; }
  /// mode actually used for the prepared sequence (Graph falls back to Eager when a host op
  /// cannot be recorded)
  ExecMode effective_mode() const { return graphExec_ ? ExecMode::Graph : ExecMode::Eager; }
  int device() const { return device_; }
  std::string device_name() const;
  /// number of top-level nodes of the compiled graph (0 in eager mode)
  size_t graph_nodes() const { return graphNodes_; }
  /// number of dependency edges of the compiled graph
  size_t graph_edges() const { return graphEdges_; }
  /// node count by type of the compiled single-iteration graph ("kernel", "host", "memcpy",
  /// "event_record", ...; empty in eager mode)
  std::map<std::string, int> graph_node_types() const;
  void set_watchdog(double s, double k = -1) {
    watchdogS_ = s;
    if (k >= 0) watchdogK_ = k;
  }
  double watchdog_floor() const { return watchdogS_; }
  double watchdog_k() const { return watchdogK_; }
  /// per-iteration seconds the watchdog expects of the prepared schedule (0: not run yet)
  double expected_iter_s() const { return expected_; }
  /// seconds the watchdog would give a run of n iterations right now
  double watchdog_budget(int64_t n) const;
  /// runs the watchdog aborted so far
  int watchdog_fired() const { return fired_.load(); }
  void set_spin_sync(bool on) { spinSync_ = on; }
  bool spin_sync() const { return spinSync_; }
  /// compile `u` consecutive iterations into one graph (amortizes the per-launch cost; the
  /// iterations stay ordered exactly as the schedule's final host syncs order them)
  void set_graph_unroll(int u);
  int graph_unroll() const { return unroll_; }

  /// One op of a traced run: GPU ops carry device times (timing events recorded around the
  /// launch on the op's stream), host ops (syncs, CPU ops) host wall-clock times; both in us
  /// from the start of the trace (the two clocks are aligned at that start only).
  struct Span {
    std::string name;
    int stream; // -1: host
    int iteration;
    double start_us, end_us;
  };
  /// Run `seq` eagerly `iterations` times with a timing event before and after every GPU op and
  /// return the per-op timeline (the mode and prepared sequence stay as they were). The events
  /// add a little issue overhead, so use this to look at a schedule, not to time it.
  std::vector<Span> trace(const Sequence &seq, int iterations = 1);

private:
  void *event(int e);
  void *internal_event();
  void destroy_graph();
  bool recordable(const Sequence &seq) const;
  void *build_graph(int iterations, size_t &nodes, size_t &edges);
  void run_impl(int64_t n);
  /// run `body` (a blocking wait on the device) under the watchdog with `budget` seconds
  void guarded(double budget, const char *what, const std::function<void()> &body);
  bool guarding_ = false; // inside guarded() (runs are issued from one thread)
  int captureAs_ = -1;    // graph build: the logical stream of the op being captured on the origin

  int device_ = 0;
  ExecMode mode_;
  std::vector<void *> streams_;
  std::vector<void *> spare_;    // never used: hardware-queue padding (pad_streams)
  int pad_ = 0;                  // streams owned at least (schedule streams + spares)
  std::vector<void *> events_;   // schedule events
  std::vector<void *> internal_; // StreamWait helpers
  void *timerEv_[2] = {nullptr, nullptr};
  size_t internalUsed_ = 0;
  Sequence seq_;
  void *graphExec_ = nullptr;  // one iteration
  void *graphExecU_ = nullptr; // unroll_ iterations
  void *graphExecR_ = nullptr; // remR_ iterations (precompile)
  int64_t remR_ = 0;
  // the source graph of every instantiated exec, destroyed together with it (not right after
  // instantiation: some HIP releases keep referring to the source graph's nodes from the exec)
  std::unordered_map<void *, void *> graphOf_;
  void destroy_exec(void *exec);
  int unroll_ = 1;
  bool spinSync_ = true;
  size_t graphNodes_ = 0, graphEdges_ = 0;
  struct Slot {
    Sequence seq;
    void *exec = nullptr, *execU = nullptr;
    size_t nodes = 0, edges = 0;
    double expected = 0;
  };
  size_t slot_ = 0; // selected slot (prepare_many)
  std::vector<Slot> slots_; // prepare_many: own the compiled graphs (graphExec_ borrows)

  double watchdogS_ = 0;
  double watchdogK_ = 50;
  // longest per-iteration seconds of a run of the prepared schedule (read by the watchdog)
  std::atomic<double> expected_{0};
  std::atomic<int> fired_{0};
  DeadlineClaim deadline_; // the current guarded wait vs the watchdog (core/deadline_claim.hpp)
  std::atomic<double> budget_{0}; // seconds the current run was given
  std::atomic<uint64_t> runGen_{0};  // runs started so far
  // communicator aborts still running on their own threads (shared: a thread may outlive this)
  std::shared_ptr<std::atomic<int>> abortsPending_ = std::make_shared<std::atomic<int>>(0);
  std::atomic<bool> stop_{false};
  std::thread watchdog_;
  bool traceOps_ = false; // TZ_TRACE=ops: name every op on stderr as eager mode issues it
};

/// Chrome trace-event JSON (chrome://tracing, Perfetto) of a traced timeline: one track per
/// stream plus a host track
Json chrome_trace(const std::vector<HipRuntime::Span> &spans);

/// How a schedule becomes a hipGraph (set_graph_capture; python: TZ_GRAPH_CAPTURE at import):
///  * Schedule (default): ONE stream capture for the whole schedule. It begins on the origin
///    stream, is forked to the other streams by an event, every op is enqueued in issue order
///    on its own stream with that stream's capture dependencies set to exactly the nodes the
///    schedule's happens-before relation implies (hipStreamUpdateCaptureDependencies), and the
///    streams are joined back to the origin before the capture ends. One capture sequence per
///    graph is the pattern NCCL-API capture is built for: RCCL keeps one persistent plan set per
///    capture id and ties its lifetime to the captured graph (which lives as long as its exec).
///  * Child ("child"): every op captured alone into a graph of its own and added as a child-graph
///    node. Kept only for A/B diagnosis: HIP runs child-graph nodes one after another, so it
///    costs all branch concurrency (profiles/archive/r3b_rccl_loopback/child_graph_overlap.jsonl).
enum class CaptureMode { Schedule, Child };
/// the mode for schedules without RCCL between ranks (default Schedule)
CaptureMode capture_mode();
/// whether a mode was forced by set_graph_capture (then it holds for every schedule, RCCL ones
/// included)
bool capture_mode_forced();
/// "schedule" or "child": force that mode for every schedule; "auto": Schedule, and for RCCL
/// schedules whatever the RCCL preflight found exact (process-wide)
void set_graph_capture(const std::string &mode);
/// the mode for schedules with RCCL ops between ranks: whichever the RCCL preflight found exact
/// on every rank (Schedule first, Child as the fallback); Schedule until a preflight sets it
CaptureMode rccl_capture_mode();
void set_rccl_capture_mode(CaptureMode m);
/// a workload's RCCL preflight has verified (and set) the capture mode: a later workload's
/// preflight must verify that same mode, not pick another (the mode is per process)
bool rccl_capture_settled();
const char *capture_mode_name(CaptureMode m);

/// Builds one hipGraph from ops enqueued on a fixed set of streams (hipStream_t as void*;
/// streams[0] is the origin). The runtime's graph build and the transports' preflights share
/// it, so a preflight tests exactly what candidates run. Schedule mode: one capture on the
/// origin; every op is enqueued there (its launch receives the capture stream) behind exactly
/// the dependencies given, so the graph has the schedule's edges and nothing else. Child mode:
/// every op captured alone on its own stream and added as a child-graph node. Not copyable; the
/// destructor abandons an unfinished build (ends the capture, destroys the partial graph).
class GraphBuilder {
public:
  GraphBuilder(const std::vector<void *> &streams, CaptureMode mode);
  ~GraphBuilder();
  GraphBuilder(const GraphBuilder &) = delete;
  GraphBuilder &operator=(const GraphBuilder &) = delete;
  /// enqueue one op of logical stream `stream` behind `deps` (hipGraphNode_t as void*):
  /// `launch(captureStream)` issues its work. Returns the op's tail nodes; empty when it
  /// enqueued nothing.
  std::vector<void *> add(int stream, const std::vector<void *> &deps,
                          const std::function<void(void *)> &launch);
  /// end the build: the caller owns the returned hipGraph_t (as void*)
  void *finish();
  CaptureMode mode() const { return mode_; }

private:
  void abandon();
  std::vector<void *> streams_;
  CaptureMode mode_;
  void *graph_ = nullptr; // Child: the graph being assembled
  bool capturing_ = false;
};

/// streams a runtime owns at least when its options say -1 (default 6; the spare ones are never
/// used: they keep hipGraph branch streams off the launch stream's hardware queue,
/// profiles/archive/r4_pad/). (A single root node per captured schedule was measured too and retired:
/// it changed neither the branch probes nor the RCCL probe, profiles/archive/r4_root/.)
int pad_streams();
/// set the default above (process-wide; python: TZ_PAD_STREAMS at import)
void set_default_pad_streams(int n);

/// route the core's trace ranges (MCTS phases, schedule ops in eager runs) to roctx
void enable_roctx(bool on);
/// hipGetDeviceCount (0 if no GPU / no driver)
int hip_device_count();
/// throw tz::Error if `err` (a hipError_t) is not success
void hip_check(int err, const char *what, const char *file, int line);

} // namespace tz

#define TZ_HIP(x) ::tz::hip_check(int(x), #x, __FILE__, __LINE__)
