// A multi-rank program through the C++ library: the native counterpart of the reference's MPI
// drivers (tenzing-mcts/examples/halo_run_strategy.hpp, whose graphs hold Isend/Irecv/Wait ops
// from include/tenzing/mpi/ops_mpi.hpp). One process per GPU, ranks on a ring:
//
//   Start -> interior ------------------------------------------> Finish
//   Start -> xfer (send my edge right, receive the left edge) -> boundary -> allreduce -> Finish
//
// `interior` is a long kernel that needs nothing from the neighbours. `xfer` is an RCCL grouped
// send/recv (SendRecvOp), `boundary` consumes what arrived, and `allreduce` sums it over all
// ranks (AllReduceOp). On one stream the communication chain waits behind the interior kernel;
// the search finds the schedule that overlaps them. Every rank benchmarks every candidate together
// and the slowest rank's time counts. The winning schedule's results are checked on every rank.
//
//   tenzing_amd/bin/tz-example-ring                                    # 1 rank (self exchange)
//   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 --no-python tenzing_amd/bin/tz-example-ring
//   mpirun -n 8 tenzing_amd/bin/tz-example-ring                        # as the reference's drivers
//
// Under torchrun, ranks come from RANK / WORLD_SIZE / LOCAL_RANK and rank 0 publishes its
// control-plane port in /tmp/tz_ring_<MASTER_PORT>; under an MPI launcher the control plane is
// MPI_COMM_WORLD. Built by `python -m tenzing_amd._build` against
// build/libtenzing_amd.a.
#include "core/solve.hpp"
#include "hip/comm_ops.hpp"
#include "hip/hip_runtime.hpp"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

namespace {

int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// y <- y + 1, `reps` times per element, on `blocks` workgroups: a long kernel that leaves most
// CUs free, so the communication chain can run beside it
__global__ void interior_k(float *y, int n, int reps) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float v = y[i];
    for (int r = 0; r < reps; ++r) v = v + 1.f;
    y[i] = v;
  }
}

// z = 2 * received edge (overwrites, so every iteration computes the same z)
__global__ void boundary_k(const float *in, float *z, int m) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) z[i] = 2.f * in[i];
}

class InteriorOp : public tz::GpuOp {
public:
  InteriorOp(float *y, int n, int reps) : y_(y), n_(n), reps_(reps) {}
  std::string name() const override { return "interior"; }
  std::string kind() const override { return "Interior"; }
  double cost_us() const override { return 60.0; }
  void launch(void *stream, tz::Executor &) const override {
    hipLaunchKernelGGL(interior_k, dim3(64), dim3(256), 0, static_cast<hipStream_t>(stream), y_, n_,
                       reps_);
  }

private:
  float *y_;
  int n_, reps_;
};

class BoundaryOp : public tz::GpuOp {
public:
  BoundaryOp(const float *in, float *z, int m) : in_(in), z_(z), m_(m) {}
  std::string name() const override { return "boundary"; }
  std::string kind() const override { return "Boundary"; }
  double cost_us() const override { return 3.0; }
  void launch(void *stream, tz::Executor &) const override {
    hipLaunchKernelGGL(boundary_k, dim3((m_ + 255) / 256), dim3(256), 0,
                       static_cast<hipStream_t>(stream), in_, z_, m_);
  }

private:
  const float *in_;
  float *z_;
  int m_;
};

} // namespace

int main() {
  int rank = env_int("RANK", 0), size = env_int("WORLD_SIZE", 1);
  int local = env_int("LOCAL_RANK", rank);
  try {
    std::shared_ptr<tz::Ctrl> ctrl;
    if (!std::getenv("WORLD_SIZE") && tz::MpiCtrl::launched()) {
      ctrl = std::make_shared<tz::MpiCtrl>();
      rank = ctrl->rank();
      size = ctrl->size();
      local = tz::MpiCtrl::launcher_local_rank() >= 0 ? tz::MpiCtrl::launcher_local_rank() : rank;
    } else if (size > 1) {
      auto t = std::make_shared<tz::TcpCtrl>(rank, size);
      const char *port = std::getenv("MASTER_PORT");
      t->rendezvous_file(std::string("/tmp/tz_ring_") + (port ? port : "default"),
                         std::getenv("MASTER_ADDR") ? std::getenv("MASTER_ADDR") : "127.0.0.1");
      ctrl = t;
    } else {
      ctrl = std::make_shared<tz::SelfCtrl>();
    }
    tz::log_rank() = rank;
    const int ndev = tz::hip_device_count();
    TZ_CHECK(ndev > 0, "no GPU visible");
    const int device = local % ndev;
    TZ_HIP(hipSetDevice(device));

    const int n = 1 << 16, reps = 1000, m = 1 << 20, streams = 2;
    float *y = nullptr, *edge = nullptr, *in = nullptr, *z = nullptr;
    TZ_HIP(hipMalloc(&y, n * sizeof(float)));
    TZ_HIP(hipMalloc(&edge, m * sizeof(float)));
    TZ_HIP(hipMalloc(&in, m * sizeof(float)));
    TZ_HIP(hipMalloc(&z, m * sizeof(float)));
    std::vector<float> h(m, float(rank + 1)); // my edge: rank + 1 everywhere
    TZ_HIP(hipMemcpy(edge, h.data(), m * sizeof(float), hipMemcpyHostToDevice));

    // one communicator per stream: RCCL matches operations per communicator in issue order
    const tz::CommSet comms = tz::make_rccl_comms(*ctrl, device, streams);
    auto interior = std::make_shared<InteriorOp>(y, n, reps);
    auto xfer = std::make_shared<tz::SendRecvOp>("xfer", comms, edge, size_t(m), (rank + 1) % size,
                                                 in, size_t(m), (rank + size - 1) % size, 0);
    auto boundary = std::make_shared<BoundaryOp>(in, z, m);
    auto allreduce = std::make_shared<tz::AllReduceOp>("allreduce", comms, z, z, size_t(m), 0);
    tz::Graph g;
    g.start_then(interior);
    g.then_finish(interior);
    g.start_then(xfer);
    g.then(xfer, boundary);
    g.then(boundary, allreduce);
    g.then_finish(allreduce);

    tz::HipRuntimeOpts ro;
    ro.device = device;
    ro.n_streams = streams;
    ro.mode = tz::ExecMode::Graph; // every candidate a hipGraph, RCCL kernels captured
    auto rt = std::make_unique<tz::HipRuntime>(ro);
    tz::MctsOpts opts;
    opts.n_iters = 20;
    opts.bench.n_iters = 5;
    opts.bench.max_retries = 1;
    opts.bench.target_secs = 0.003;
    tz::SearchResult res;
    {
      tz::EmpiricalBenchmarker bench(*rt, *ctrl);
      res = tz::mcts_explore(g, tz::Platform::make_n_streams(streams), bench, *ctrl, opts);
    }
    const int b = res.best();
    double worst = 0;
    for (const auto &s : res.sims) worst = std::max(worst, s.res.pct10);
    const tz::Sequence &best = res.sims[size_t(b)].seq;
    int interior_stream = -1, xfer_stream = -1;
    for (const auto &e : best.entries) {
      auto gb = std::dynamic_pointer_cast<const tz::BoundGpuOp>(e.op);
      if (!gb) continue;
      if (gb->name() == "interior") interior_stream = gb->stream();
      if (gb->name() == "xfer") xfer_stream = gb->stream();
    }

    // the winning schedule computes what the program says: 3 iterations from zero
    TZ_HIP(hipMemset(y, 0, n * sizeof(float)));
    TZ_HIP(hipMemset(z, 0, m * sizeof(float)));
    TZ_HIP(hipDeviceSynchronize()); // the schedule's streams are non-blocking
    rt->prepare(best);
    rt->run(3);
    rt->device_sync();
    std::vector<float> hy(n), hz(m);
    TZ_HIP(hipMemcpy(hy.data(), y, n * sizeof(float), hipMemcpyDeviceToHost));
    TZ_HIP(hipMemcpy(hz.data(), z, m * sizeof(float), hipMemcpyDeviceToHost));
    const float wy = 3.f * reps, wz = float(size) * float(size + 1); // sum over ranks of 2(r+1)
    double bad = 0;
    for (int i = 0; i < n; ++i) bad += hy[i] != wy;
    for (int i = 0; i < m; ++i) bad += hz[i] != wz;
    ctrl->allreduce_sum(&bad, 1);
    if (rank == 0)
      std::cout << "{\"ranks\": " << size << ", \"candidates\": " << res.sims.size()
                << ", \"best_us\": " << res.sims[size_t(b)].res.pct10 * 1e6
                << ", \"worst_us\": " << worst * 1e6 << ", \"interior_stream\": " << interior_stream
                << ", \"xfer_stream\": " << xfer_stream << ", \"bad\": " << int64_t(bad)
                << ", \"best\": " << best.json().dump() << "}\n";
    rt.reset(); // streams go before the communicators and buffers they use
    (void)hipFree(y);
    (void)hipFree(edge);
    (void)hipFree(in);
    (void)hipFree(z);
    return bad == 0 ? 0 : 1;
  } catch (const std::exception &e) {
    std::cerr << "[rank " << rank << "] " << e.what() << "\n";
    return 2;
  }
}
