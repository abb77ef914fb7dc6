// Numeric helpers and the measurement-noise randomness test.
//
// Parity: reference include/tenzing/numeric.hpp:18-107 (avg/med/var/stddev/corr),
// src/numeric.cpp:11-42 (prime_factors, round_up), src/randomness.cpp:12-63 (Wald-Wolfowitz
// runs test + compound_test). The reference runs test reports "reject" whenever either half has
// fewer than 10 samples (randomness.cpp:30-32), which forces every benchmark with nIters < 20 to
// exhaust its retries; here that behaviour is explicit: `RunsTestSmall::Reject` reproduces it,
// `RunsTestSmall::Accept` (the default) treats too-small samples as not testable.
#pragma once

#include <cmath>
#include <cstdint>
#include <vector>

namespace tz {

double avg(const std::vector<double> &v);
double med(std::vector<double> v);
double var(const std::vector<double> &v);
double stddev(const std::vector<double> &v);
template <typename T> double corr(const std::vector<T> &a, const std::vector<T> &b);

/// prime factors of n in descending order (reference numeric.cpp:11-31)
std::vector<int64_t> prime_factors(int64_t n);
int64_t round_up(int64_t x, int64_t step);

/// percentile by nearest-rank on a sorted copy: v[size * pct / 100]
double percentile_sorted(const std::vector<double> &sorted, int pct);

enum class RunsTestSmall { Accept, Reject };
/// true if the sequence is judged NON-random (reject) at alpha=0.05
bool runs_test(const std::vector<double> &v, RunsTestSmall small = RunsTestSmall::Accept);
bool compound_test(const std::vector<double> &v, RunsTestSmall small = RunsTestSmall::Accept);

// ---- template implementation
template <typename T> double corr(const std::vector<T> &a, const std::vector<T> &b) {
  const size_t n = a.size() < b.size() ? a.size() : b.size();
  if (n == 0) return 0;
  double ma = 0, mb = 0;
  for (size_t i = 0; i < n; ++i) {
    ma += double(a[i]);
    mb += double(b[i]);
  }
  ma /= n;
  mb /= n;
  double sab = 0, saa = 0, sbb = 0;
  for (size_t i = 0; i < n; ++i) {
    const double da = double(a[i]) - ma, db = double(b[i]) - mb;
    sab += da * db;
    saa += da * da;
    sbb += db * db;
  }
  if (saa == 0 || sbb == 0) return 0;
  return sab / (std::sqrt(saa) * std::sqrt(sbb));
}

} // namespace tz
