#!/usr/bin/env python3
"""Search how to overlap gradient all-reduces with backward GEMMs (data parallel, 1-8 GPUs).

A toy backward pass of `--layers` layers, each one a bf16 GEMM on the matrix cores (torch.matmul
-> hipBLASLt) that produces that layer's gradient bucket. Every bucket is summed over the ranks
with an `AllReduceOp` (RCCL over xGMI), then one fused update applies all buckets. The GEMMs form
a chain (backward order); bucket i can be reduced once GEMM i is done. MCTS chooses the issue
order, the stream of every GEMM and every all-reduce, and the sync placement. With several
ranks, the fast schedules put the all-reduces on their own stream, behind the next GEMMs. On one
GPU the all-reduces are local copies, so there the search mostly shows its own overhead.

  python examples/grad_allreduce_overlap.py [--iters 40]
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/grad_allreduce_overlap.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd import parallel  # noqa: E402
from tenzing_amd.ops import comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--n", type=int, default=4096, help="GEMM size; one bucket = n*n bf16")
    ap.add_argument("--streams", type=int, default=2)
    a = ap.parse_args()

    ctrl, dev = parallel.init()
    torch.cuda.set_device(dev)
    d = torch.device("cuda", dev)
    torch.manual_seed(ctrl.rank)
    act = [torch.randn(a.n, a.n, device=d, dtype=torch.bfloat16) for _ in range(a.layers + 1)]
    grad = [torch.empty(a.n, a.n, device=d, dtype=torch.bfloat16) for _ in range(a.layers)]
    red = [torch.empty_like(x) for x in grad]
    params = torch.zeros(a.layers, a.n, a.n, device=d, dtype=torch.bfloat16)
    comms = tz._tz.make_rccl_comms(ctrl, dev, a.streams)

    def on(stream_ptr, fn):
        with torch.cuda.stream(torch.cuda.ExternalStream(stream_ptr)):
            fn()

    g = tz.Graph()
    prev = None
    update = tz.PyGpuOp("update", lambda s: on(s, lambda: [params[i].add_(red[i], alpha=-1e-3)
                                                         for i in range(a.layers)]), 50.0, False)
    for i in reversed(range(a.layers)):  # backward: last layer first
        gemm = tz.PyGpuOp(f"bwd{i}", (lambda i: lambda s: on(
            s, lambda: torch.matmul(act[i].t(), act[i + 1], out=grad[i])))(i), 200.0, False)
        ar = comm.all_reduce(f"allreduce{i}", comms, grad[i], red[i])
        if prev is None:
            g.start_then(gemm)
        else:
            g.then(prev, gemm)
        g.then(gemm, ar)
        g.then(ar, update)
        prev = gemm
    g.then(prev, update)
    g.then_finish(update)

    rt = tz.HipRuntime(device=dev, n_streams=a.streams, watchdog_s=120.0)
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    opts = tz.MctsOpts()
    opts.n_iters = a.iters
    opts.bench = tz.BenchOpts(n_iters=5, max_retries=1, target_secs=0.01)
    res = tz.mcts_explore(g, tz.Platform(a.streams), bench, ctrl, opts)
    if ctrl.rank == 0:
        times = sorted((s.res.pct10, i) for i, s in enumerate(res.sims))
        best, worst = res.sims[times[0][1]], res.sims[times[-1][1]]

        def streams(seq):
            return {e["name"]: e.get("stream") for e in json.loads(seq.json())
                    if e["name"].startswith(("bwd", "allreduce"))}

        print(json.dumps({"ranks": ctrl.size, "candidates": len(res.sims),
                          "best_ms": best.res.pct10 * 1e3, "worst_ms": worst.res.pct10 * 1e3,
                          "best_streams": streams(best.seq), "search_wall_s": res.wall_s}))
    torch.cuda.synchronize()
    del bench, rt
    return 0


if __name__ == "__main__":
    sys.exit(main())
