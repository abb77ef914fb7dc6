#include "benchmark.hpp"
#include "util.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace tz {

Json BenchResult::json() const {
  Json j;
  j["pct01"] = pct01;
  j["pct10"] = pct10;
  j["pct50"] = pct50;
  j["pct90"] = pct90;
  j["pct99"] = pct99;
  j["stddev"] = stddev;
  j["samples_per_measurement"] = samples_per_measurement;
  j["retries"] = retries;
  return j;
}

BenchResult BenchResult::from_times(std::vector<double> times) {
  BenchResult r;
  if (times.empty()) return r;
  r.stddev = ::tz::stddev(times);
  std::sort(times.begin(), times.end());
  r.pct01 = percentile_sorted(times, 1);
  r.pct10 = percentile_sorted(times, 10);
  r.pct50 = percentile_sorted(times, 50);
  r.pct90 = percentile_sorted(times, 90);
  r.pct99 = percentile_sorted(times, 99);
  return r;
}

Json BenchOpts::json() const {
  Json j;
  j["nIters"] = n_iters;
  j["maxRetries"] = max_retries;
  j["targetSecs"] = target_secs;
  if (device_timer) j["deviceTimer"] = true;
  if (race_ratio > 0) j["raceRatio"] = race_ratio;
  if (settle_ratio > 0) j["settleRatio"] = settle_ratio;
  return j;
}

// ---------------------------------------------------------------- Empirical

EmpiricalBenchmarker::EmpiricalBenchmarker(ExecutorRunner &runner, Ctrl &ctrl)
    : runner_(runner), ctrl_(ctrl) {}

EmpiricalBenchmarker::Measurement EmpiricalBenchmarker::measure(int64_t nHint, double targetSecs,
                                                                bool deviceTimer) {
  Measurement m{std::max<int64_t>(1, nHint), 0};
  while (true) {
    // the control plane waits in the max-reduction below for the slowest rank's run: never give
    // up on it before that run's own watchdog would
    const double budget = runner_.run_budget(m.n);
    if (budget > 0) ctrl_.ensure_timeout(budget + 60.0);
    ctrl_.barrier();
    const double t0 = wtime();
    // a run-time failure (launch error, watchdog, op check) may hit one rank only: it travels
    // with the time in the same max-reduction, so every rank throws together and the next
    // collective still matches
    std::string err;
    double dev = -1.0;
    try {
      if (deviceTimer) dev = runner_.run_device_timed(m.n);
      else runner_.run(m.n);
    } catch (const std::exception &e) {
      err = e.what();
    }
    double red[2] = {dev >= 0 ? dev : wtime() - t0, err.empty() ? 0.0 : 1.0};
    ctrl_.allreduce_max(red, 2); // "true" time is the max over ranks
    if (red[1] != 0.0)
      throw CandidateFailed("schedule run failed" +
                            (err.empty() ? std::string(" on another rank") : ": " + err));
    const double elapsed = red[0];
    if (elapsed < targetSecs) {
      const double perSample = std::max(elapsed / double(m.n), 1e-9);
      const double est = targetSecs / perSample * 1.1;
      // a batch that ran for an eighth of the target or more is long enough to time, so it
      // sizes the next batch directly (the 10 % margin lands it past the target); a shorter
      // one is dominated by launch latency and grows 8x at most. A candidate is sized in ~3
      // runs (about 1.3x the target) instead of ~6 runs (about 4.5x) when closing half the gap
      // per run (the round-1 rule, retired after its A/B)
      const int64_t jump = int64_t(std::ceil(est));
      m.n = elapsed >= targetSecs / 8 ? jump : std::min(jump, m.n * 8);
      m.n = std::max<int64_t>(m.n, 1);
      const int64_t k = std::max<int64_t>(1, runner_.batch_multiple());
      m.n = (m.n + k - 1) / k * k;
    } else {
      m.time = elapsed / double(m.n);
      return m;
    }
  }
}

void EmpiricalBenchmarker::collective_prepare(const std::function<void()> &fn) {
  // preparation (event provisioning, hipGraph compilation) is local and may fail on one rank
  // only; every rank must then leave together instead of entering mismatched collectives
  std::string err;
  try {
    fn();
  } catch (const std::exception &e) {
    err = e.what();
  }
  double bad = err.empty() ? 0.0 : 1.0;
  if (ctrl_.size() > 1) ctrl_.allreduce_max(&bad, 1);
  if (bad != 0.0)
    throw CandidateFailed("schedule preparation failed" +
                          (err.empty() ? std::string(" on another rank") : ": " + err));
}

BenchResult EmpiricalBenchmarker::benchmark(const Sequence &seq, const BenchOpts &opts) {
  collective_prepare([&] { runner_.prepare(seq); });
  std::vector<double> times;
  int retries = 0;
  int64_t hint = 1;
  bool settled = false;
  for (int left = opts.max_retries; opts.max_retries == 0 || left > 0; --left) {
    Measurement m = measure(1, opts.target_secs, opts.device_timer); // warm-up, size the batch
    hint = m.n;
    times.clear();
    bool raced = false;
    settled = false;
    for (int64_t i = 0; i < opts.n_iters; ++i) {
      m = measure(hint, opts.target_secs, opts.device_timer);
      hint = std::max(hint, m.n);
      times.push_back(m.time);
      if (opts.race_ratio > 0 && best_ > 0 && int64_t(times.size()) >= opts.race_min &&
          i + 1 < opts.n_iters &&
          *std::min_element(times.begin(), times.end()) > opts.race_ratio * best_) {
        raced = true; // clearly slower than the best so far: enough to rank it
        break;
      }
      if (opts.settle_ratio > 0 && int64_t(times.size()) >= std::max(2, opts.settle_min) &&
          i + 1 < opts.n_iters) {
        const auto mm = std::minmax_element(times.begin(), times.end());
        if (*mm.second - *mm.first <= opts.settle_ratio * *mm.first) {
          settled = true; // the samples agree: further ones would not change its ranking
          ++settled_;
          break;
        }
      }
    }
    if (raced) {
      ++raced_;
      break;
    }
    if (settled) break; // consistent samples: no randomness retry needed
    // per-measurement times are already maxed across ranks inside measure()
    if (compound_test(times, opts.small_sample) && left > 1) {
      ++retries;
      if (ctrl_.rank() == 0) TZ_LOG(Info, "failed randomness test (" << left - 1 << " left)");
      continue;
    }
    break;
  }
  BenchResult r = BenchResult::from_times(times);
  r.samples_per_measurement = hint;
  r.retries = retries;
  if ((settled || int64_t(times.size()) == opts.n_iters) && (best_ == 0.0 || r.pct10 < best_))
    best_ = r.pct10;
  return r;
}

std::vector<BenchResult> EmpiricalBenchmarker::benchmark_many(const std::vector<Sequence> &seqs,
                                                              const BenchOpts &opts, uint64_t seed) {
  const size_t k = seqs.size();
  std::vector<BenchResult> out(k);
  if (k == 0) return out;
  collective_prepare([&] { runner_.prepare_many(seqs); });
  // warm each schedule up and size its batch once
  std::vector<int64_t> hint(k, 1);
  for (size_t i = 0; i < k; ++i) {
    runner_.select(i);
    hint[i] = measure(1, opts.target_secs, opts.device_timer).n;
  }
  std::vector<std::vector<double>> times(k);
  std::mt19937_64 rng(seed + 0x5EEDull);
  std::vector<int> perm(k);
  for (int64_t it = 0; it < std::max<int64_t>(1, opts.n_iters); ++it) {
    std::string msg;
    if (ctrl_.rank() == 0) {
      for (size_t i = 0; i < k; ++i) perm[i] = int(i);
      std::shuffle(perm.begin(), perm.end(), rng);
      msg.assign(reinterpret_cast<const char *>(perm.data()), k * sizeof(int));
    }
    ctrl_.bcast(msg, 0);
    TZ_CHECK(msg.size() == k * sizeof(int), "permutation broadcast truncated");
    std::memcpy(perm.data(), msg.data(), msg.size());
    for (int i : perm) {
      runner_.select(size_t(i));
      Measurement m = measure(hint[size_t(i)], opts.target_secs, opts.device_timer);
      hint[size_t(i)] = std::max(hint[size_t(i)], m.n);
      times[size_t(i)].push_back(m.time);
    }
  }
  for (size_t i = 0; i < k; ++i) {
    out[i] = BenchResult::from_times(times[i]);
    out[i].samples_per_measurement = hint[i];
  }
  return out;
}

void HostExecutor::run(int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    for (const auto &e : seq_.entries) e.op->run(*this);
}

// ---------------------------------------------------------------- Sim

SimExecutor::SimExecutor(int nStreams, SimParams p)
    : n_(nStreams), p_(p), rng_(p.seed), streamFree_(nStreams, 0.0), lastEnd_(nStreams, 0.0),
      pending_(nStreams), used_(nStreams, 0) {}

void SimExecutor::graph_dep(int stream, double t) {
  // work the stream's own order already covers costs nothing; an event from the sequence's
  // start (t = 0) neither
  if (t > lastEnd_[stream] && t > 0) pending_[stream].push_back(t);
}

double SimExecutor::dur(double us) {
  if (p_.noise <= 0) return us;
  std::normal_distribution<double> nd(1.0, p_.noise);
  return std::max(0.0, us * nd(rng_));
}

double SimParams::rate_GBps(const std::string &engine) const {
  const auto it = engine_GBps.find(engine);
  TZ_CHECK(it != engine_GBps.end() && it->second > 0, "sim: no rate for engine '" << engine << "'");
  return it->second;
}

double SimParams::capacity_GBps(const std::string &resource) const {
  auto it = resource_GBps.find(resource);
  if (it == resource_GBps.end()) it = resource_GBps.find(resource.substr(0, resource.find(':')));
  TZ_CHECK(it != resource_GBps.end() && it->second > 0, "sim: no capacity for resource '" << resource << "'");
  return it->second;
}

double SimExecutor::link_duration(const GpuOp &op, double start) {
  const std::vector<Traffic> tr = op.traffic();
  // bytes per (resource, engine): an op that sends several boxes to one peer is one transfer
  std::map<std::pair<std::string, std::string>, double> per;
  for (const Traffic &t : tr)
    if (t.bytes > 0) per[{t.resource, t.engine}] += t.bytes;
  // A transfer shares its resource with the transfers whose [start, end) overlaps its own.
  // Ops are simulated in program order, not in start-time order (an op issued earlier on another
  // stream may start later), so every interval is kept and tested for overlap; the op's own
  // end depends on how many it shares with, so the estimate is refined once (alone -> with the
  // overlaps of that window -> with the overlaps of the longer window).
  auto duration = [&](double window) {
    double slowest = 0;
    for (const auto &kv : per) {
      int k = 0;
      for (const auto &iv : active_[kv.first.first]) k += iv.first < start + window && iv.second > start;
      const double rate = std::min(p_.rate_GBps(kv.first.second),
                                   p_.capacity_GBps(kv.first.first) / double(k + 1));
      slowest = std::max(slowest, kv.second / (rate * 1e3)); // GB/s = 1e3 bytes per us
    }
    return op.latency_us() + slowest;
  };
  double est = duration(0.0); // (window 0: nothing overlaps an empty window)
  est = duration(est);
  est = duration(est);
  const double d = dur(est);
  for (const auto &kv : per) active_[kv.first.first].push_back({start, start + d});
  return d;
}

void SimExecutor::launch(const GpuOp &op, int stream) {
  TZ_CHECK(stream >= 0 && stream < n_, "sim stream out of range");
  double start;
  if (p_.graph) {
    graph_dep(stream, host_); // after a host sync or host op: a dependency like any other
    start = streamFree_[stream];
    std::vector<double> &pw = pending_[stream];
    if (!pw.empty()) {
      const double last = *std::max_element(pw.begin(), pw.end());
      start = std::max(start, last + p_.graph_join_us + p_.graph_wait_us * double(pw.size() - 1));
      pw.clear();
    }
  } else {
    host_ += p_.launch_us;
    start = std::max(host_, streamFree_[stream]);
  }
  double d;
  if (p_.link_model && !op.traffic().empty()) {
    d = link_duration(op, start);
  } else {
    int busy = 0;
    for (int s = 0; s < n_; ++s)
      if (s != stream && streamFree_[s] > start) ++busy;
    d = dur(op.cost_us()) * (1.0 + p_.contention * busy);
  }
  lastEnd_[stream] = start + d;
  used_[stream] = 1;
  streamFree_[stream] = start + d + (p_.graph ? p_.graph_gap_us : 0.0);
  trace_.push_back({op.name(), stream, start, start + d});
}

void SimExecutor::event_record(int event, int stream) {
  if (event >= int(events_.size())) events_.resize(event + 1, 0.0);
  if (p_.graph) {
    double t = lastEnd_[stream];
    for (double w : pending_[stream]) t = std::max(t, w);
    events_[event] = t;
    return;
  }
  host_ += p_.api_us;
  events_[event] = std::max(streamFree_[stream], host_);
}

void SimExecutor::stream_wait_event(int stream, int event) {
  if (p_.graph) {
    if (event < int(events_.size())) graph_dep(stream, events_[event]);
    return;
  }
  host_ += p_.api_us;
  if (event < int(events_.size()))
    streamFree_[stream] = std::max(streamFree_[stream], events_[event]);
}

void SimExecutor::event_sync(int event) {
  if (p_.graph) {
    if (event < int(events_.size())) host_ = std::max(host_, events_[event]);
    return;
  }
  if (event < int(events_.size()) && events_[event] > host_) host_ = events_[event] + p_.sync_us;
  else host_ += p_.api_us;
}

void SimExecutor::stream_sync(int stream) {
  if (p_.graph) {
    host_ = std::max(host_, lastEnd_[stream]);
    return;
  }
  if (streamFree_[stream] > host_) host_ = streamFree_[stream] + p_.sync_us;
  else host_ += p_.api_us;
}

void SimExecutor::stream_wait(int waiter, int waitee) {
  if (p_.graph) {
    graph_dep(waiter, lastEnd_[waitee]);
    return;
  }
  host_ += 2 * p_.api_us;
  streamFree_[waiter] = std::max(streamFree_[waiter], streamFree_[waitee]);
}

void SimExecutor::device_sync() {
  if (p_.graph) {
    for (double t : lastEnd_) host_ = std::max(host_, t);
    return;
  }
  double m = host_;
  for (double t : streamFree_) m = std::max(m, t);
  host_ = m + p_.sync_us;
}

double SimExecutor::run_once(const Sequence &seq) {
  host_ = 0;
  std::fill(streamFree_.begin(), streamFree_.end(), 0.0);
  std::fill(lastEnd_.begin(), lastEnd_.end(), 0.0);
  std::fill(used_.begin(), used_.end(), 0);
  for (auto &pw : pending_) pw.clear();
  events_.assign(events_.size(), 0.0);
  trace_.clear();
  active_.clear();
  for (const auto &e : seq.entries) e.op->run(*this);
  if (p_.graph) {
    // replayed back to back: the next iteration starts after the join of every stream used
    double end = host_;
    int used = 0;
    for (int s = 0; s < n_; ++s) {
      end = std::max(end, lastEnd_[s]);
      used += used_[s];
    }
    if (used > 1) end += p_.graph_join_us + p_.graph_wait_us * double(used - 2);
    else if (used == 1) end += p_.graph_gap_us;
    return end;
  }
  // the sequence ends host-synchronized with all its GPU work (Finish has GPU preds synced)
  double end = host_;
  for (double t : streamFree_) end = std::max(end, t);
  return end;
}

BenchResult SimBenchmarker::benchmark(const Sequence &seq, const BenchOpts &opts) {
  SimParams p = p_;
  p.seed = rng_();
  SimExecutor ex(n_, p);
  std::vector<double> times;
  const int64_t n = std::max<int64_t>(1, std::min<int64_t>(opts.n_iters, 200));
  for (int64_t i = 0; i < n; ++i) times.push_back(ex.run_once(seq) * 1e-6);
  if (ctrl_ && ctrl_->size() > 1) ctrl_->allreduce_max(times.data(), times.size()); // max over ranks
  BenchResult r = BenchResult::from_times(times);
  r.samples_per_measurement = 1;
  return r;
}

// ---------------------------------------------------------------- CSV replay

static std::vector<std::string> split_top(const std::string &line, char delim) {
  // split on delim, but not inside JSON strings
  std::vector<std::string> out;
  std::string cur;
  bool inStr = false, esc = false;
  for (char c : line) {
    if (inStr) {
      cur.push_back(c);
      if (esc) esc = false;
      else if (c == '\\') esc = true;
      else if (c == '"') inStr = false;
      continue;
    }
    if (c == '"') inStr = true;
    if (c == delim) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

CsvBenchmarker::CsvBenchmarker(const std::string &path, const Graph &g) {
  std::ifstream f(path);
  TZ_CHECK(f, "cannot open " << path);
  OpIndex idx(g);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty() || line[0] == '{' || line[0] == '#') continue; // opts header / comments
    auto cols = split_top(line, '|');
    if (cols.size() < 7) continue;
    BenchResult r;
    try {
      r.pct01 = std::stod(cols[1]);
      r.pct10 = std::stod(cols[2]);
      r.pct50 = std::stod(cols[3]);
      r.pct90 = std::stod(cols[4]);
      r.pct99 = std::stod(cols[5]);
      r.stddev = std::stod(cols[6]);
    } catch (...) {
      continue; // header row
    }
    Sequence s;
    for (size_t i = 7; i < cols.size(); ++i) s.push_back(idx.from_json(Json::parse(cols[i])));
    data_.emplace(s.canonical_key(), r);
  }
}

BenchResult CsvBenchmarker::benchmark(const Sequence &seq, const BenchOpts &) {
  auto it = data_.find(seq.canonical_key());
  if (it == data_.end()) TZ_THROW("no equivalent CSV data for sequence " << seq.desc());
  return it->second;
}

BenchResult CachingBenchmarker::benchmark(const Sequence &seq, const BenchOpts &opts) {
  const std::string k = seq.canonical_key();
  auto it = cache_.find(k);
  if (it != cache_.end()) {
    ++hits_;
    return it->second;
  }
  BenchResult r = inner_.benchmark(seq, opts);
  cache_.emplace(k, r);
  return r;
}

std::string csv_row(size_t i, const BenchResult &r, const Sequence &seq) {
  std::ostringstream ss;
  ss.precision(9);
  ss << i << "|" << r.pct01 << "|" << r.pct10 << "|" << r.pct50 << "|" << r.pct90 << "|"
     << r.pct99 << "|" << r.stddev;
  for (const auto &e : seq.entries) ss << "|" << e.op->json().dump();
  return ss.str();
}

} // namespace tz
