// The handoff between a guarded wait (a run of a schedule, a device synchronization) and the
// watchdog thread that may abort it. Host-only, so the race between "the run finishes at its
// deadline" and "the watchdog fires" is unit-tested without a GPU (tz-unit, also under TSan).
//
// One atomic double carries the whole protocol: > 0 is the armed deadline, 0 means no wait, and
// two sentinels mark an aborted wait. The watchdog claims an expired wait with one CAS; the
// waiter ends its wait with one exchange. Exactly one of them sees the other: a wait that ends
// at its deadline is either claimed (the waiter sees kClaimed and reports the abort) or not
// (the CAS fails and the watchdog fires nothing). No device abort or communicator abort can hit
// a wait that already returned as a success.
#pragma once

#include <atomic>

namespace tz {

class DeadlineClaim {
public:
  static constexpr double kClaimed = -1;  // the watchdog claimed the wait (set by its CAS only)
  static constexpr double kDraining = -2; // the claimed wait returned and drains the device

  /// waiter: arm a wait that must end by `deadline` (seconds on the wtime() clock)
  void arm(double deadline) { d_.store(deadline); }
  /// watchdog: claim the wait if it is armed and past its deadline; true if this call claimed
  /// it (then, and only then, the watchdog aborts the device waits)
  bool try_claim(double now) {
    double d = d_.load();
    if (d <= 0 || now <= d) return false;
    return d_.compare_exchange_strong(d, kClaimed);
  }
  /// waiter: the wait ended. True if the watchdog had claimed it: the state is then kDraining
  /// until drained(); false otherwise (the state is back to 0)
  bool finish() {
    // claimed -> draining in one step: the watchdog never sees 0 in between, so a drain that
    // then hangs still counts as a pending abort (its grace exit stays armed)
    double c = kClaimed;
    if (d_.compare_exchange_strong(c, kDraining)) return true;
    // not claimed: back to 0, unless the watchdog claims it right now (then drain after all)
    double d = d_.load();
    while (d != kClaimed) {
      if (d_.compare_exchange_weak(d, 0)) return false;
    }
    c = kClaimed;
    return d_.compare_exchange_strong(c, kDraining);
  }
  /// waiter: the aborted wait has drained
  void drained() { d_.store(0); }
  /// watchdog: a claimed wait has not come back yet (still blocked, or draining)
  bool abort_pending() const {
    const double d = d_.load();
    return d == kClaimed || d == kDraining;
  }
  double value() const { return d_.load(); }

private:
  std::atomic<double> d_{0};
};

} // namespace tz
