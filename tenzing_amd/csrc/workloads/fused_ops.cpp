// Ops that run two workloads' GPU work in one launch (horizontal fusion).
//
// Not in the reference: its SpMV and halo graphs only share streams. On one GPU the halo's
// direct moves are bound by HBM and the SpMV's local product by its L2 gathers; launched on two
// streams of one schedule they pay a fork / join per iteration, and back to back they add up
// (profiles/r6_negative/). One kernel that interleaves the two kinds of workgroups runs them at
// once without the join (kern::box_move_spmv).
#include "workloads.hpp"

#include "core/util.hpp"

#include <algorithm>

namespace tz {

namespace {

class MoveSpmv : public GpuOp {
public:
  MoveSpmv(std::shared_ptr<const HaloExchange> h, std::vector<int> dirs, std::shared_ptr<const DistSpmv> s,
           std::string name, int lanes, bool intoY)
      : h_(std::move(h)), dirs_(std::move(dirs)), s_(std::move(s)), name_(std::move(name)), lanes_(lanes),
        intoY_(intoY) {
    TZ_CHECK(lanes_ > kern::kSpmvIlp && lanes_ <= kern::kSpmvIlp + 4 && (lanes_ - kern::kSpmvIlp) != 3,
             name_ << ": lanes must be kSpmvIlp + 1, 2 or 4");
    for (int i : dirs_) TZ_CHECK(h_->is_direct(i), name_ << ": direction " << i << " is not a self move");
    TZ_CHECK(int(dirs_.size()) <= kern::kMaxBoxes, name_ << ": at most " << kern::kMaxBoxes << " directions");
  }
  std::string name() const override { return name_; }
  std::string kind() const override { return "MoveSpmv"; }
  double move_bytes() const {
    double b = 0;
    for (int i : dirs_) b += 2.0 * 8.0 * double(h_->box_elems(i));
    return b;
  }
  double spmv_bytes() const { return 12.0 * double(s_->local_nnz()) + 8.0 * double(s_->local_rows()); }
  // the simulator: both at once (a move-bound launch plus part of the SpMV's latency)
  double cost_us() const override {
    const double mv = 3.0 + move_bytes() / 5.0e6, sp = 4.0 + spmv_bytes() / 3.0e6;
    return std::max(mv, sp) + 0.5 * std::min(mv, sp);
  }
  std::vector<Traffic> traffic() const override { return {{"hbm", "kernel", move_bytes() + spmv_bytes()}}; }
  double latency_us() const override { return 3.0; }
  void launch(void *s, Executor &) const override {
    const std::vector<kern::MoveDesc> ms = h_->direct_moves(dirs_);
    TZ_CHECK(int(ms.size()) <= kern::kMaxBoxes, name_ << ": too many moves for one launch");
    kern::box_move_spmv(ms.data(), int(ms.size()), s_->local_job(lanes_, intoY_), s);
  }

private:
  std::shared_ptr<const HaloExchange> h_;
  std::vector<int> dirs_;
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
  int lanes_;
  bool intoY_;
};

} // namespace

std::shared_ptr<GpuOp> make_move_spmv_op(std::shared_ptr<const HaloExchange> h, std::vector<int> dirs,
                                         std::shared_ptr<const DistSpmv> s, std::string name, int lanes,
                                         bool intoY) {
  return std::make_shared<MoveSpmv>(std::move(h), std::move(dirs), std::move(s), std::move(name), lanes, intoY);
}

} // namespace tz
