#!/usr/bin/env python3
"""Cost of cross-stream dependencies on the MI355X: time every schedule of a small op chain
(each op a fixed-duration busy kernel) in eager and graph mode. Same-stream edges are free
(in-queue ordering); cross-stream edges cost an event record + wait (eager) or a cross-queue
barrier packet (graph), which this measures.

  python scripts/depcost.py --ops 4 --us 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=4)
    ap.add_argument("--us", type=float, default=20.0)
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--unroll", type=int, default=10)
    ap.add_argument("--max-seqs", type=int, default=64)
    a = ap.parse_args()

    import tenzing_amd as tz

    g = tz.Graph()
    ops = [tz.BusyKernelOp(f"k{i}", a.us, a.blocks) for i in range(a.ops)]
    g.start_then(ops[0])
    for x, y in zip(ops, ops[1:]):
        g.then(x, y)
    g.then_finish(ops[-1])
    seqs = tz.get_all_sequences(g, tz.Platform(2), max_seqs=a.max_seqs)
    rt = tz.HipRuntime(device=0, n_streams=2, graph_unroll=a.unroll)
    for seq in seqs:
        streams = [o.stream for o in seq.ops() if isinstance(o, tz._tz.BoundGpuOp)]
        crossings = sum(1 for x, y in zip(streams, streams[1:]) if x != y)
        row = {"streams": streams, "cross": crossings, "syncs": seq.count_sync_ops()}
        for name, m in (("eager", tz.ExecMode.Eager), ("graph", tz.ExecMode.Graph)):
            rt.set_mode(m)
            rt.prepare(seq)
            rt.run(20)
            t0 = time.perf_counter()
            rt.run(a.iters)
            rt.device_sync()
            row[name + "_us"] = round((time.perf_counter() - t0) / a.iters * 1e6, 2)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
