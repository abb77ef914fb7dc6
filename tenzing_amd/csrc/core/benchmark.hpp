// Benchmarkers: turn a Sequence into a timing distribution.
//
// Parity: reference include/tenzing/benchmarker.hpp:14-30 (Result pct01..pct99/stddev, Opts
// nIters/maxRetries), src/benchmarker.cpp:83-167 (EmpiricalBenchmarker: adaptive batching to a
// target wall time, barrier, max over ranks, runs-test retries, percentiles) and :169-223
// (CsvBenchmarker replay). Additions: SimBenchmarker (discrete-event model of streams, events and
// the host thread; hardware-free solver tests and what-if searches), a HostExecutor for CPU-only
// sequences, measurement caching by canonical schedule key.
#pragma once

#include "ctrl.hpp"
#include "numeric.hpp"
#include "serdes.hpp"
#include "state.hpp"

#include <functional>
#include <map>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace tz {

struct BenchResult {
  double pct01 = 0, pct10 = 0, pct50 = 0, pct90 = 0, pct99 = 0, stddev = 0;
  int64_t samples_per_measurement = 0;
  int retries = 0;
  Json json() const;
  static BenchResult from_times(std::vector<double> times);
};

struct BenchOpts {
  int64_t n_iters = 1000;      // measurements per benchmark (reference Opts::nIters)
  int max_retries = 10;        // runs-test retries (reference Opts::maxRetries)
  double target_secs = 0.01;   // each measurement batches runs to at least this wall time
  RunsTestSmall small_sample = RunsTestSmall::Accept;
  // time each measurement with device events around the batch (GPU time, no host issue or
  // wake-up latency) when the runner has them; false: host wall clock, like the reference
  bool device_timer = false;
  // racing: once `race_min` measurements of a candidate are all slower than race_ratio x the
  // best pct10 this benchmarker has seen, stop measuring it (a search only needs to know it is
  // bad). 0 = off. Every rank sees the same max-over-ranks times, so all stop together.
  double race_ratio = 0.0;
  int race_min = 2;
  // settling: once `settle_min` measurements of a candidate all lie within settle_ratio of
  // each other ((max - min) / min), stop: more samples would not move its percentiles by more
  // than that. 0 = off. The decision uses max-over-ranks times, so all ranks stop together.
  double settle_ratio = 0.0;
  int settle_min = 4;
  Json json() const;
};

class Benchmarker {
public:
  virtual ~Benchmarker() = default;
  virtual BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) = 0;
};

/// Runs sequences on an Executor (the HIP runtime, or HostExecutor) with host wall-clock timing,
/// max across ranks of the control plane.
class ExecutorRunner {
public:
  virtual ~ExecutorRunner() = default;
  /// provision per-sequence resources (events, captured graphs)
  virtual void prepare(const Sequence &seq) = 0;
  /// run the prepared sequence `n` times back to back (host returns when all work is done)
  virtual void run(int64_t n) = 0;
  /// provision several sequences at once; select(k) makes the k-th the one run() executes
  /// (interleaved benchmarking). Default: re-prepare on every select.
  virtual void prepare_many(const std::vector<Sequence> &seqs) { many_ = seqs; }
  virtual void select(size_t k) { prepare(many_.at(k)); }
  /// runners with a device clock: run `n` times and return the device time in seconds
  /// between an event before the first op and one after the last (or < 0 if unsupported)
  virtual double run_device_timed(int64_t n) {
    run(n);
    return -1.0;
  }
  /// batch sizes that run without a remainder (a compiled graph of K unrolled iterations: K),
  /// so a measurement times the same launches as a long run does
  virtual int64_t batch_multiple() const { return 1; }
  /// the longest a run of `n` iterations may take before the runner gives up on it (its
  /// watchdog budget plus grace), 0 if unbounded: every rank's collectives around a run must
  /// wait at least that long for the slowest rank
  virtual double run_budget(int64_t n) const {
    (void)n;
    return 0.0;
  }

private:
  std::vector<Sequence> many_;
};

class EmpiricalBenchmarker : public Benchmarker {
public:
  EmpiricalBenchmarker(ExecutorRunner &runner, Ctrl &ctrl);
  BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) override;
  /// Several schedules measured interleaved (reference src/benchmarker.cpp:21-76): every
  /// iteration runs each schedule once (one batched measurement) in a random order chosen by
  /// rank 0 and broadcast, so slow drift (clocks, thermals, other tenants) spreads evenly over
  /// the schedules instead of biasing whichever ran last. Times are max over ranks.
  std::vector<BenchResult> benchmark_many(const std::vector<Sequence> &seqs, const BenchOpts &opts,
                                          uint64_t seed = 0);
  /// candidates cut short by racing so far
  int64_t raced() const { return raced_; }
  /// candidates whose measurements agreed early (settle_ratio) so far
  int64_t settled() const { return settled_; }
  /// forget the best time racing compares against
  void reset_race() { best_ = 0.0; }

private:
  struct Measurement {
    int64_t n;
    double time;
  };
  Measurement measure(int64_t nHint, double targetSecs, bool deviceTimer = false);
  void collective_prepare(const std::function<void()> &fn);
  ExecutorRunner &runner_;
  Ctrl &ctrl_;
  double best_ = 0.0; // best complete pct10 seen (racing); identical on every rank
  int64_t raced_ = 0;
  int64_t settled_ = 0;
};

/// Host-only executor: GPU ops are launched with a null stream, synchronously (tests/CPU runs).
class HostExecutor : public ExecutorRunner, public Executor {
public:
  explicit HostExecutor(int nStreams) : n_(nStreams) {}
  int num_streams() const override { return n_; }
  void launch(const GpuOp &op, int) override { op.launch(nullptr, *this); }
  void event_record(int, int) override {}
  void stream_wait_event(int, int) override {}
  void event_sync(int) override {}
  void stream_sync(int) override {}
  void stream_wait(int, int) override {}
  void device_sync() override {}
  void prepare(const Sequence &seq) override { seq_ = seq; }
  void run(int64_t n) override;

private:
  int n_;
  Sequence seq_;
};

/// Discrete-event model: each stream executes its ops in order, a GPU op starts no earlier than
/// the host issues it, events carry completion times, host syncs block the host clock.
struct SimParams {
  double launch_us = 4.0;   // host cost to issue a kernel / comm op
  double api_us = 1.0;      // host cost of an event record / stream wait
  double sync_us = 5.0;     // host wake-up latency after a blocking sync
  double noise = 0.0;       // relative gaussian noise on each op duration
  uint64_t seed = 0;
  /// concurrent kernels share the device: when k GPU ops overlap, each runs at rate
  /// 1/(1 + contention*(k-1)); 0 = perfect overlap
  double contention = 0.0;
  /// Link-aware model: a GPU op that reports traffic() takes latency_us() plus, over its
  /// resources, the longest bytes / rate, where rate = min(engine rate, resource capacity /
  /// (transfers active on that resource when it starts + 1)). Ops without traffic keep cost_us().
  bool link_model = false;
  /// GB/s one transfer of an engine reaches alone (kernel: a local HBM stream; put / wide:
  /// kernel stores over one xGMI link at the default / wide workgroup count; sdma / memcpy: copy
  /// engines; rccl: an RCCL send; host: stores into host memory over PCIe)
  std::map<std::string, double> engine_GBps = {{"kernel", 5000.0}, {"put", 60.0},  {"wide", 90.0},
                                               {"sdma", 50.0},     {"memcpy", 50.0}, {"rccl", 50.0},
                                               {"host", 40.0}};
  /// capacity of a resource class (the text before ':') or of one resource ("xgmi:3")
  std::map<std::string, double> resource_GBps = {{"hbm", 5000.0}, {"xgmi", 120.0}, {"pcie", 50.0}};
  /// hipGraph replay, the mode the bench searches and times in: no host issue cost (launch_us
  /// and api_us unused); consecutive ops on one stream are graph_gap_us apart; an op that waits
  /// on work of other streams starts graph_join_us after the latest of it, plus graph_wait_us
  /// per further dependency; an iteration ends with the join of every stream it used (one gap
  /// if it used one). Calibrated on MI355X from device timestamps of unrolled fork/join graphs
  /// (scripts/stagger_probe.hip, profiles/r5_branch/README.md): 1.0 / 5.5 / 1.2 us.
  bool graph = false;
  double graph_gap_us = 1.0;
  double graph_join_us = 5.5;
  double graph_wait_us = 1.2;
  double rate_GBps(const std::string &engine) const;
  double capacity_GBps(const std::string &resource) const;
};

class SimExecutor : public Executor {
public:
  SimExecutor(int nStreams, SimParams p);
  int num_streams() const override { return n_; }
  void launch(const GpuOp &op, int stream) override;
  void host_busy(double us) override { host_ += us; }
  bool simulated() const override { return true; }
  void event_record(int event, int stream) override;
  void stream_wait_event(int stream, int event) override;
  void event_sync(int event) override;
  void stream_sync(int stream) override;
  void stream_wait(int waiter, int waitee) override;
  void device_sync() override;
  /// simulated wall time (us) of one run of the sequence, starting from an idle machine
  double run_once(const Sequence &seq);
  /// trace of (op name, stream, start, end) of the last run
  struct Span {
    std::string name;
    int stream;
    double start, end;
  };
  const std::vector<Span> &trace() const { return trace_; }

private:
  double dur(double us);
  /// duration of a GPU op starting at `start` under the link-aware model (registers its
  /// transfers as active on their resources until start + duration)
  double link_duration(const GpuOp &op, double start);
  /// graph mode: wait (on the device) for work that ends at `t` before the next op of `stream`
  void graph_dep(int stream, double t);
  int n_;
  SimParams p_;
  std::mt19937_64 rng_;
  double host_ = 0;
  std::vector<double> streamFree_;
  // resource -> [start, end) of every transfer of this run on it
  std::map<std::string, std::vector<std::pair<double, double>>> active_;
  std::vector<double> events_;
  std::vector<Span> trace_;
  // graph mode: end of each stream's last op, its pending cross-stream dependencies, and
  // whether the iteration used it
  std::vector<double> lastEnd_;
  std::vector<std::vector<double>> pending_;
  std::vector<char> used_;
};

class SimBenchmarker : public Benchmarker {
public:
  /// `ctrl` (optional): every rank simulates its own graph's copy of the sequence and the
  /// result is the max over ranks, as the empirical benchmarker's is (SPMD searches on CPUs)
  SimBenchmarker(int nStreams, SimParams p, Ctrl *ctrl = nullptr)
      : n_(nStreams), p_(p), rng_(p.seed + 17), ctrl_(ctrl) {}
  BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) override;

private:
  int n_;
  SimParams p_;
  std::mt19937_64 rng_;
  Ctrl *ctrl_ = nullptr;
};

/// Replays recorded timings from a results CSV (`i|p01|p10|p50|p90|p99|stddev|op-json|...`),
/// matching sequences by equivalence (reference CsvBenchmarker, src/benchmarker.cpp:169-223).
class CsvBenchmarker : public Benchmarker {
public:
  CsvBenchmarker(const std::string &path, const Graph &g);
  BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) override;
  size_t size() const { return data_.size(); }

private:
  std::unordered_map<std::string, BenchResult> data_;
};

/// Wraps another benchmarker and returns cached results for equivalent sequences.
class CachingBenchmarker : public Benchmarker {
public:
  explicit CachingBenchmarker(Benchmarker &inner) : inner_(inner) {}
  BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) override;
  size_t hits() const { return hits_; }

private:
  Benchmarker &inner_;
  std::unordered_map<std::string, BenchResult> cache_;
  size_t hits_ = 0;
};

/// one row of the reference results CSV
std::string csv_row(size_t i, const BenchResult &r, const Sequence &seq);

} // namespace tz
