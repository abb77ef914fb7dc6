// Operation IR: graph vertices, bound (executable) operations and synchronization operations.
//
// Parity map (reference -> here):
//   OpBase (include/tenzing/operation.hpp:64-86)          -> OpBase (stable string kind tags
//                                                            instead of typeid hash ordering)
//   ChoiceOp (:90-93), CompoundOp (operation_compound.hpp) -> ChoiceOp, CompoundOp
//   BoundOp::run(Platform&) (:96-99), CpuOp (:102-103)     -> BoundOp::run(Executor&), CpuOp
//   Start/Finish/NoOp (:114-157)                           -> Start/Finish/NoOp
//   GpuOp::run(cudaStream_t), BoundGpuOp (cuda/ops_cuda.hpp:194-238)
//                                                          -> GpuOp::launch(hipStream_t,...),
//                                                             BoundGpuOp
//   CudaEventRecord / CudaStreamWaitEvent / CudaEventSync / StreamWait / StreamSync
//   (cuda/ops_cuda.hpp:37-190)                             -> EventRecord / StreamWaitEvent /
//                                                             EventSync / StreamWait / StreamSync
// The synchronization ops are executor-agnostic: they call Executor virtuals, so the same
// sequence runs on the HIP runtime (hipEventRecord/hipStreamWaitEvent/...), inside a hipGraph
// capture, or in the discrete-event simulator. Their JSON "kind" strings keep the reference's
// schedule schema so schedules interoperate with tenzing CSV tooling.
#pragma once

#include "json.hpp"

#include <memory>
#include <string>
#include <vector>

namespace tz {

class Executor;
class Graph;

enum class OpClass {
  Start,    // graph source, host no-op
  Finish,   // graph sink, host no-op
  Cpu,      // executed by the control thread (NoOp, user host ops, host transports)
  Gpu,      // must be bound to a stream before it can execute
  BoundGpu, // a Gpu op + stream
  Sync,     // event record / wait / host sync inserted by the synchronizer
  Compound, // a sub-graph, expanded by an Expand decision
  Choice,   // alternative implementations, resolved by a Choose decision
};

const char *op_class_name(OpClass c);

class OpBase {
public:
  virtual ~OpBase() = default;
  /// unique name within a graph (the serialization key)
  virtual std::string name() const = 0;
  /// stable type tag, used in JSON and equality
  virtual std::string kind() const = 0;
  virtual OpClass op_class() const = 0;
  /// JSON description; default {"name": name()} (reference operation.cpp:12-16)
  virtual Json json() const;
  virtual std::string desc() const { return name(); }
  /// value equality (defaults to same kind and name)
  virtual bool eq(const OpBase &o) const { return kind() == o.kind() && name() == o.name(); }
  /// cost-model hint for the simulator, microseconds (device time for GPU ops, host time for
  /// CPU ops)
  virtual double cost_us() const { return 0.0; }
  /// in-flight bytes this op moves (for reporting)
  virtual double bytes() const { return 0.0; }
  /// Ordering domain. Ops that share a non-empty domain run in one total order: each happens
  /// after the previous op of its domain in the schedule, an implicit graph edge that the
  /// synchronizer covers with events like any other edge (State::domain_pred) and that verify()
  /// checks. RCCL ops use "rccl". Every rank runs the same schedule, so every device then sees
  /// the communication ops in the same order, one at a time. NCCL-API semantics promise no
  /// progress for concurrent operations on different communicators, so leaving two of them
  /// unordered could deadlock the ranks.
  virtual std::string order_domain() const { return {}; }

  bool is_bound() const;
  bool is_cpu_like() const; // Start, Finish, Cpu, Sync
};

using OpPtr = std::shared_ptr<const OpBase>;

/// an op the control thread can execute right now
class BoundOp : public OpBase {
public:
  virtual void run(Executor &ex) const = 0;
};
using BoundOpPtr = std::shared_ptr<const BoundOp>;

/// host-executed operation
class CpuOp : public BoundOp {
public:
  OpClass op_class() const override { return OpClass::Cpu; }
};

class Start : public CpuOp {
public:
  std::string name() const override { return "Start"; }
  std::string kind() const override { return "Start"; }
  OpClass op_class() const override { return OpClass::Start; }
  void run(Executor &) const override {}
};

class Finish : public CpuOp {
public:
  std::string name() const override { return "Finish"; }
  std::string kind() const override { return "Finish"; }
  OpClass op_class() const override { return OpClass::Finish; }
  void run(Executor &) const override {}
};

class NoOp : public CpuOp {
public:
  explicit NoOp(std::string name, double cost_us = 0) : name_(std::move(name)), cost_(cost_us) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "NoOp"; }
  Json json() const override;
  double cost_us() const override { return cost_; }
  void run(Executor &ex) const override;

private:
  std::string name_;
  double cost_;
};

/// Host op that sleeps: a hardware-free timing model for solver tests (the reference's legacy
/// tenzing-mcts/src_mcts_test/mcts.cpp:23-67 SlowFirst/FastFirst sleep ops).
class SleepOp : public CpuOp {
public:
  SleepOp(std::string name, double us) : name_(std::move(name)), us_(us) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SleepOp"; }
  double cost_us() const override { return us_; }
  void run(Executor &) const override;

private:
  std::string name_;
  double us_;
};

/// Bytes an op moves through one shared resource, for the simulator's link-aware cost model
/// (SimParams::link_model): `resource` is what concurrent ops share ("hbm", "xgmi:<peer rank>",
/// "pcie"), `engine` what moves the bytes ("kernel", "put", "wide", "sdma", "memcpy", "rccl",
/// "host"), which caps the rate one transfer gets.
struct Traffic {
  std::string resource;
  std::string engine;
  double bytes = 0;
};

/// GPU work that has to be bound to a stream. Implementations enqueue on `stream`
/// (a hipStream_t, passed as void* so this header stays HIP-free).
class GpuOp : public OpBase {
public:
  OpClass op_class() const override { return OpClass::Gpu; }
  virtual void launch(void *stream, Executor &ex) const = 0;
  /// true if the op can be recorded into a hipGraph by stream capture
  virtual bool capturable() const { return true; }
  /// the bytes this op moves through shared resources (empty: the simulator uses cost_us())
  virtual std::vector<Traffic> traffic() const { return {}; }
  /// fixed time beside the traffic (launch, signalling), for the link-aware model
  virtual double latency_us() const { return 4.0; }
};
using GpuOpPtr = std::shared_ptr<const GpuOp>;

/// GPU op that only models time (simulation / tests). On a real executor it launches nothing.
class SimGpuOp : public GpuOp {
public:
  /// `traffic` (optional): what it moves under the link-aware model, which then takes
  /// `us` as its fixed latency instead of its whole cost
  SimGpuOp(std::string name, double us, std::string domain = "", std::vector<Traffic> traffic = {})
      : name_(std::move(name)), us_(us), domain_(std::move(domain)), traffic_(std::move(traffic)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SimGpuOp"; }
  double cost_us() const override { return us_; }
  std::string order_domain() const override { return domain_; }
  void launch(void *, Executor &) const override {}
  std::vector<Traffic> traffic() const override { return traffic_; }
  double latency_us() const override { return us_; }

private:
  std::string name_;
  double us_;
  std::string domain_;
  std::vector<Traffic> traffic_;
};

class BoundGpuOp : public BoundOp {
public:
  BoundGpuOp(GpuOpPtr op, int stream) : op_(std::move(op)), stream_(stream) {}
  std::string name() const override { return op_->name(); }
  std::string kind() const override { return op_->kind(); }
  OpClass op_class() const override { return OpClass::BoundGpu; }
  Json json() const override; // inner json + {"stream": s} (reference ops_cuda.cpp:199-203)
  std::string desc() const override;
  bool eq(const OpBase &o) const override;
  double cost_us() const override { return op_->cost_us(); }
  double bytes() const override { return op_->bytes(); }
  std::string order_domain() const override { return op_->order_domain(); }
  void run(Executor &ex) const override;

  const GpuOpPtr &unbound() const { return op_; }
  int stream() const { return stream_; }

private:
  GpuOpPtr op_;
  int stream_;
};

/// base of synchronizer-generated ops
class SyncOp : public BoundOp {
public:
  OpClass op_class() const override { return OpClass::Sync; }
  std::string name() const override { return name_; }
  void set_name(std::string n) { name_ = std::move(n); }
  bool eq(const OpBase &o) const override; // by kind + fields, names ignored

  virtual int stream() const { return -1; }
  virtual int event() const { return -1; }
  virtual int stream2() const { return -1; }

protected:
  std::string name_;
};

/// hipEventRecord(event, stream)  — JSON kind "CudaEventRecord" (schema compatibility)
class EventRecord : public SyncOp {
public:
  EventRecord(int event, int stream, std::string name = "");
  std::string kind() const override { return "CudaEventRecord"; }
  Json json() const override;
  std::string desc() const override;
  void run(Executor &ex) const override;
  int stream() const override { return stream_; }
  int event() const override { return event_; }

private:
  int event_, stream_;
};

/// hipStreamWaitEvent(stream, event) — JSON kind "CudaStreamWaitEvent"
class StreamWaitEvent : public SyncOp {
public:
  StreamWaitEvent(int stream, int event, std::string name = "");
  std::string kind() const override { return "CudaStreamWaitEvent"; }
  Json json() const override;
  std::string desc() const override;
  void run(Executor &ex) const override;
  int stream() const override { return stream_; }
  int event() const override { return event_; }

private:
  int stream_, event_;
};

/// hipEventSynchronize(event) — JSON kind "CudaEventSync"
class EventSync : public SyncOp {
public:
  explicit EventSync(int event, std::string name = "");
  std::string kind() const override { return "CudaEventSync"; }
  Json json() const override;
  std::string desc() const override;
  void run(Executor &ex) const override;
  int event() const override { return event_; }

private:
  int event_;
};

/// hipStreamSynchronize(stream) — JSON kind "StreamSync"
class StreamSync : public SyncOp {
public:
  explicit StreamSync(int stream, std::string name = "");
  std::string kind() const override { return "StreamSync"; }
  Json json() const override;
  std::string desc() const override;
  void run(Executor &ex) const override;
  int stream() const override { return stream_; }

private:
  int stream_;
};

/// waiter stream waits for all work currently in waitee (record + wait on an internal event)
/// — JSON kind "StreamWait" (reference ops_cuda.hpp:37-74)
class StreamWait : public SyncOp {
public:
  StreamWait(int waiter, int waitee, std::string name = "");
  std::string kind() const override { return "StreamWait"; }
  Json json() const override;
  std::string desc() const override;
  void run(Executor &ex) const override;
  int stream() const override { return waiter_; }
  int stream2() const override { return waitee_; }

private:
  int waiter_, waitee_;
};

/// an op that is itself a sub-graph (reference operation_compound.hpp:8-13)
class CompoundOp : public OpBase {
public:
  OpClass op_class() const override { return OpClass::Compound; }
  virtual std::shared_ptr<const Graph> graph() const = 0;
};

/// alternative implementations of one vertex (reference operation.hpp:90-93)
class ChoiceOp : public OpBase {
public:
  OpClass op_class() const override { return OpClass::Choice; }
  virtual std::vector<OpPtr> choices() const = 0;
};

/// simple ChoiceOp holding a fixed list
class StaticChoiceOp : public ChoiceOp {
public:
  StaticChoiceOp(std::string name, std::vector<OpPtr> choices)
      : name_(std::move(name)), choices_(std::move(choices)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "ChoiceOp"; }
  std::vector<OpPtr> choices() const override { return choices_; }

private:
  std::string name_;
  std::vector<OpPtr> choices_;
};

/// simple CompoundOp holding a fixed graph
class StaticCompoundOp : public CompoundOp {
public:
  StaticCompoundOp(std::string name, std::shared_ptr<const Graph> g)
      : name_(std::move(name)), g_(std::move(g)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "CompoundOp"; }
  std::shared_ptr<const Graph> graph() const override { return g_; }

private:
  std::string name_;
  std::shared_ptr<const Graph> g_;
};

/// Runtime that executes bound ops: the HIP runtime (hip/executor), the discrete-event
/// simulator (core/sim), or a host-only executor. Reference: Platform (platform.hpp:147-219)
/// doubled as this; here the search-time platform model and the runtime are separate.
class Executor {
public:
  virtual ~Executor() = default;
  virtual int num_streams() const = 0;
  /// enqueue a GPU op on logical stream `stream`
  virtual void launch(const GpuOp &op, int stream) = 0;
  /// the control thread is busy for `us` microseconds (real executors spin, simulators
  /// advance the host clock)
  virtual void host_busy(double us);
  virtual void event_record(int event, int stream) = 0;
  virtual void stream_wait_event(int stream, int event) = 0;
  virtual void event_sync(int event) = 0;
  virtual void stream_sync(int stream) = 0;
  virtual void stream_wait(int waiter, int waitee) = 0;
  virtual void device_sync() = 0;
  /// a cost model, not a machine: ops with side effects outside the executor (host transfers
  /// over the control plane, user callbacks) only charge their cost_us() to host_busy
  virtual bool simulated() const { return false; }
  /// native handle (hipStream_t) of a logical stream, or nullptr when simulated
  virtual void *native_stream(int stream) { (void)stream; return nullptr; }
  /// logical index of a native stream handle (-1 if it is not one of this executor's)
  virtual int stream_index(const void *native) const { (void)native; return -1; }
};

} // namespace tz
