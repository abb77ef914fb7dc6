// Using tenzing-amd as a C++ library (the way the reference's drivers use tenzing-core, e.g.
// tenzing-mcts/examples/halo_run_strategy.hpp): define your own GPU op around your own HIP
// kernel, put it in an op graph, and let the MCTS solver find the best multi-stream schedule.
//
// Two independent chains, each of two small kernels that occupy only a slice of the GPU:
//   Start -> a1 -> a2 -> Finish,  Start -> b1 -> b2 -> Finish
// On one stream the chains serialize; the search should put them on different streams.
//
//   tenzing_amd/bin/tz-example-custom-op            # on the GPU
//   tenzing_amd/bin/tz-example-custom-op --sim      # discrete-event model, no GPU
//
// Built by `python -m tenzing_amd._build` against build/libtenzing_amd.a.
#include "core/solve.hpp"
#include "hip/hip_runtime.hpp"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <vector>

namespace {

// y = a * y + b, repeated `reps` times per element (a small, latency-bound kernel: `blocks`
// workgroups leave most of the 256 CUs free for a concurrent stream)
__global__ void affine_k(float *y, int n, float a, float b, int reps) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float v = y[i];
    for (int r = 0; r < reps; ++r) v = a * v + b;
    y[i] = v;
  }
}

class AffineOp : public tz::GpuOp {
public:
  AffineOp(std::string name, float *y, int n, float a, float b, int reps, int blocks)
      : name_(std::move(name)), y_(y), n_(n), a_(a), b_(b), reps_(reps), blocks_(blocks) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "Affine"; }
  double cost_us() const override { return 40.0; } // hint for the simulator
  void launch(void *stream, tz::Executor &) const override {
    hipLaunchKernelGGL(affine_k, dim3(blocks_), dim3(256), 0, static_cast<hipStream_t>(stream), y_,
                       n_, a_, b_, reps_);
  }

private:
  std::string name_;
  float *y_;
  int n_;
  float a_, b_;
  int reps_, blocks_;
};

} // namespace

int main(int argc, char **argv) {
  const bool sim = argc > 1 && !std::strcmp(argv[1], "--sim");
  const int n = 1 << 16, reps = 2000, blocks = 64;
  float *ya = nullptr, *yb = nullptr;
  if (!sim) {
    TZ_HIP(hipSetDevice(0));
    TZ_HIP(hipMalloc(&ya, n * sizeof(float)));
    TZ_HIP(hipMalloc(&yb, n * sizeof(float)));
  }
  // chain a: y <- 1*y + 1 (twice per iteration); chain b: y <- 1*y + 2
  auto a1 = std::make_shared<AffineOp>("a1", ya, n, 1.f, 1.f, reps, blocks);
  auto a2 = std::make_shared<AffineOp>("a2", ya, n, 1.f, 1.f, reps, blocks);
  auto b1 = std::make_shared<AffineOp>("b1", yb, n, 1.f, 2.f, reps, blocks);
  auto b2 = std::make_shared<AffineOp>("b2", yb, n, 1.f, 2.f, reps, blocks);
  tz::Graph g;
  g.start_then(a1);
  g.then(a1, a2);
  g.then_finish(a2);
  g.start_then(b1);
  g.then(b1, b2);
  g.then_finish(b2);

  tz::SelfCtrl ctrl;
  tz::MctsOpts opts;
  opts.n_iters = 24;
  opts.bench.n_iters = 5;
  opts.bench.max_retries = 1;
  opts.bench.target_secs = 0.005;
  const tz::Platform plat = tz::Platform::make_n_streams(2);
  tz::SearchResult res;
  std::unique_ptr<tz::HipRuntime> rt;
  if (sim) {
    tz::SimBenchmarker bench(2, tz::SimParams{});
    res = tz::mcts_explore(g, plat, bench, ctrl, opts);
  } else {
    tz::HipRuntimeOpts ro;
    ro.device = 0;
    ro.n_streams = 2;
    rt = std::make_unique<tz::HipRuntime>(ro);
    tz::EmpiricalBenchmarker bench(*rt, ctrl);
    res = tz::mcts_explore(g, plat, bench, ctrl, opts);
  }
  const int b = res.best();
  double worst = 0;
  for (const auto &s : res.sims) worst = std::max(worst, s.res.pct10);
  const tz::Sequence &best = res.sims[size_t(b)].seq;
  std::cout << "{\"candidates\": " << res.sims.size() << ", \"best_us\": " << res.sims[size_t(b)].res.pct10 * 1e6
            << ", \"worst_us\": " << worst * 1e6 << ", \"best\": " << best.json().dump() << "}\n";

  if (!sim) {
    // the winning schedule computes what the program says: 3 iterations from zero
    TZ_HIP(hipMemset(ya, 0, n * sizeof(float)));
    TZ_HIP(hipMemset(yb, 0, n * sizeof(float)));
    TZ_HIP(hipDeviceSynchronize()); // the schedule's streams are non-blocking
    rt->prepare(best);
    rt->run(3);
    rt->device_sync();
    std::vector<float> ha(n), hb(n);
    TZ_HIP(hipMemcpy(ha.data(), ya, n * sizeof(float), hipMemcpyDeviceToHost));
    TZ_HIP(hipMemcpy(hb.data(), yb, n * sizeof(float), hipMemcpyDeviceToHost));
    const float wa = 3 * 2 * reps * 1.f, wb = 3 * 2 * reps * 2.f;
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += (ha[i] != wa) + (hb[i] != wb);
    rt.reset();
    (void)hipFree(ya);
    (void)hipFree(yb);
    if (bad) {
      std::cerr << bad << " wrong elements\n";
      return 1;
    }
  }
  return 0;
}
