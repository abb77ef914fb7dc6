#include "numeric.hpp"
#include "util.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace tz {

LogLevel g_log_level = [] {
  const char *e = std::getenv("TZ_LOG");
  if (!e) return LogLevel::Warn;
  std::string s(e);
  if (s == "error") return LogLevel::Error;
  if (s == "info") return LogLevel::Info;
  if (s == "debug") return LogLevel::Debug;
  return LogLevel::Warn;
}();
LogLevel log_level() { return g_log_level; }

TraceHooks &trace_hooks() {
  static TraceHooks h;
  return h;
}
void set_log_level(LogLevel lvl) { g_log_level = lvl; }
int &log_rank() {
  static int r = 0;
  return r;
}
std::mutex &log_mutex() {
  static std::mutex m;
  return m;
}

double avg(const std::vector<double> &v) {
  if (v.empty()) return 0;
  double s = 0;
  for (double x : v) s += x;
  return s / v.size();
}

double med(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  if (n % 2) return v[n / 2];
  return 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

double var(const std::vector<double> &v) {
  if (v.size() < 2) return 0;
  const double m = avg(v);
  double s = 0;
  for (double x : v) s += (x - m) * (x - m);
  return s / (v.size() - 1);
}

double stddev(const std::vector<double> &v) { return std::sqrt(var(v)); }

std::vector<int64_t> prime_factors(int64_t n) {
  std::vector<int64_t> r;
  if (n < 2) return r;
  for (int64_t p = 2; p * p <= n; ++p) {
    while (n % p == 0) {
      r.push_back(p);
      n /= p;
    }
  }
  if (n > 1) r.push_back(n);
  std::sort(r.begin(), r.end(), std::greater<int64_t>());
  return r;
}

int64_t round_up(int64_t x, int64_t step) { return (x + step - 1) / step * step; }

double percentile_sorted(const std::vector<double> &sorted, int pct) {
  if (sorted.empty()) return 0;
  size_t i = sorted.size() * size_t(pct) / 100;
  if (i >= sorted.size()) i = sorted.size() - 1;
  return sorted[i];
}

bool runs_test(const std::vector<double> &v, RunsTestSmall small) {
  const double median = med(v);
  std::vector<int> deltas;
  deltas.reserve(v.size());
  size_t n1 = 0, n2 = 0;
  for (double t : v) {
    if (t >= median) {
      deltas.push_back(1);
      ++n1;
    } else {
      deltas.push_back(0);
      ++n2;
    }
  }
  if (n1 < 10 || n2 < 10) return small == RunsTestSmall::Reject;

  size_t nRuns = 1;
  for (size_t i = 0; i + 1 < deltas.size(); ++i) nRuns += deltas[i] != deltas[i + 1];

  const double dn1 = double(n1), dn2 = double(n2);
  const double rBar = 2 * dn1 * dn2 / (dn1 + dn2) + 1;
  const double s = std::sqrt(2 * dn1 * dn2 * (2 * dn1 * dn2 - dn1 - dn2) /
                             ((dn1 + dn2) * (dn1 + dn2) * (dn1 + dn2 - 1)));
  if (s == 0) return false;
  const double z = std::abs((double(nRuns) - rBar) / s);
  return z > 1.96;
}

bool compound_test(const std::vector<double> &v, RunsTestSmall small) {
  return runs_test(v, small);
}

} // namespace tz
