// Error macros, levelled logging, counters, timing.
//
// Parity: reference include/tenzing/macro_at.hpp:17-37 (THROW_RUNTIME, rank-prefixed STDERR),
// include/tenzing/counters.hpp:26-34 (compile-time phase counters). Differences: logging is
// levelled and runtime-controlled (env TZ_LOG=error|warn|info|debug) instead of always-on,
// and the rank prefix comes from tz::log_rank() (set by the control plane) rather than an MPI
// query, so the core has no MPI dependency.
#pragma once

#include <chrono>
#include <cstdint>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>

namespace tz {

enum class LogLevel : int { Error = 0, Warn = 1, Info = 2, Debug = 3 };

LogLevel log_level();
void set_log_level(LogLevel lvl);
int &log_rank();
std::mutex &log_mutex();

inline double wtime() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

struct Error : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

/// A candidate schedule failed on at least one rank and every rank of the control plane knows it
/// (the benchmarker agreed on the failure through a collective before throwing). Only this error
/// is safe to skip in a multi-rank search: any other exception may be local to one rank, which
/// would leave the other ranks inside mismatched collectives.
struct CandidateFailed : public Error {
  using Error::Error;
};

/// Accumulating named phase timers (reference counters::Mcts SELECT_TIME etc.).
struct Counters {
  std::map<std::string, double> seconds;
  std::map<std::string, uint64_t> counts;
  void add(const std::string &k, double s) {
    seconds[k] += s;
    counts[k] += 1;
  }
  void clear() {
    seconds.clear();
    counts.clear();
  }
};

/// RAII timer that adds its lifetime into a Counters entry.
/// Optional trace-range hooks. The core stays free of ROCm dependencies; the HIP layer installs
/// roctx push/pop here (env TZ_TRACE=roctx), so rocprofv3 --marker-trace shows MCTS phases and
/// schedule ops as named ranges next to the kernels.
struct TraceHooks {
  void (*push)(const char *) = nullptr;
  void (*pop)() = nullptr;
};
TraceHooks &trace_hooks();

struct TraceRange {
  bool on;
  explicit TraceRange(const char *name) : on(trace_hooks().push != nullptr) {
    if (on) trace_hooks().push(name);
  }
  ~TraceRange() {
    if (on) trace_hooks().pop();
  }
  TraceRange(const TraceRange &) = delete;
  TraceRange &operator=(const TraceRange &) = delete;
};

struct ScopedTimer {
  Counters &c;
  std::string key;
  double t0;
  TraceRange range;
  ScopedTimer(Counters &c_, std::string k)
      : c(c_), key(std::move(k)), t0(wtime()), range(key.c_str()) {}
  ~ScopedTimer() { c.add(key, wtime() - t0); }
};

} // namespace tz

#define TZ_THROW(msg)                                                                              \
  do {                                                                                             \
    std::ostringstream tz_ss_;                                                                     \
    tz_ss_ << __FILE__ << ":" << __LINE__ << ": " << msg;                                          \
    throw ::tz::Error(tz_ss_.str());                                                               \
  } while (0)

#define TZ_CHECK(cond, msg)                                                                        \
  do {                                                                                             \
    if (!(cond)) TZ_THROW("check failed: " #cond ": " << msg);                                     \
  } while (0)

#define TZ_LOG(lvl, msg)                                                                           \
  do {                                                                                             \
    if (int(::tz::LogLevel::lvl) <= int(::tz::log_level())) {                                      \
      std::ostringstream tz_ss_;                                                                   \
      tz_ss_ << "[tz r" << ::tz::log_rank() << " " #lvl "] " << msg << "\n";                       \
      std::lock_guard<std::mutex> tz_lk_(::tz::log_mutex());                                      \
      std::cerr << tz_ss_.str();                                                                   \
    }                                                                                              \
  } while (0)
