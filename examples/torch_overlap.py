#!/usr/bin/env python3
"""Search the schedule of a small PyTorch program on one MI355X.

The program has two independent chains:
  * gemm (bf16 8192^3 on the matrix cores, via hipBLASLt) -> row sums,
  * a 64 MiB host-to-device copy from pinned memory -> an elementwise scale.

Every op is a `tz.PyGpuOp`. Its Python callable launches torch work on the HIP stream the
schedule binds it to. MCTS explores issue order, stream binding (2 streams) and sync placement.
It should find that putting the copy chain on the other stream overlaps the DMA with the GEMM.

  python examples/torch_overlap.py [--iters 30]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--copy-mib", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    A = torch.randn(a.n, a.n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(a.n, a.n, device=dev, dtype=torch.bfloat16)
    C = torch.empty(a.n, a.n, device=dev, dtype=torch.bfloat16)
    rows = torch.empty(a.n, device=dev, dtype=torch.float32)
    host = torch.randn(a.copy_mib * 2**20 // 4, dtype=torch.float32).pin_memory()
    D = torch.empty(host.numel(), device=dev, dtype=torch.float32)

    def on(stream_ptr, fn):
        with torch.cuda.stream(torch.cuda.ExternalStream(stream_ptr)):
            fn()

    ops = {
        "gemm": lambda s: on(s, lambda: torch.matmul(A, B, out=C)),
        "rowsum": lambda s: on(s, lambda: torch.sum(C, dim=1, dtype=torch.float32, out=rows)),
        "h2d": lambda s: on(s, lambda: D.copy_(host, non_blocking=True)),
        "scale": lambda s: on(s, lambda: D.mul_(2.0)),
    }
    g = tz.Graph()
    o = {k: tz.PyGpuOp(k, fn, 100.0, False) for k, fn in ops.items()}
    g.start_then(o["gemm"])
    g.then(o["gemm"], o["rowsum"])
    g.then_finish(o["rowsum"])
    g.start_then(o["h2d"])
    g.then(o["h2d"], o["scale"])
    g.then_finish(o["scale"])

    ctrl = tz.SelfCtrl()
    rt = tz.HipRuntime(device=0, n_streams=2, watchdog_s=60.0)
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    opts = tz.MctsOpts()
    opts.n_iters = a.iters
    opts.bench = tz.BenchOpts(n_iters=5, max_retries=1, target_secs=0.01)
    res = tz.mcts_explore(g, tz.Platform(2), bench, ctrl, opts)
    times = sorted((s.res.pct10, i) for i, s in enumerate(res.sims))
    best, worst = res.sims[times[0][1]], res.sims[times[-1][1]]

    def streams(seq):
        return {e["name"]: e.get("stream") for e in json.loads(seq.json()) if e["name"] in ops}

    out = {"candidates": len(res.sims), "best_ms": best.res.pct10 * 1e3,
           "worst_ms": worst.res.pct10 * 1e3, "best_streams": streams(best.seq),
           "worst_streams": streams(worst.seq), "search_wall_s": res.wall_s}
    print(json.dumps(out))
    # the pinned-memory allocator recorded events on the schedule's streams (the async copy):
    # release that memory while the runtime, which owns the streams, is still alive
    del host
    torch.cuda.synchronize()
    if hasattr(torch._C, "_host_emptyCache"):
        torch._C._host_emptyCache()
    del bench, rt
    return 0


if __name__ == "__main__":
    sys.exit(main())
