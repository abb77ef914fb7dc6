#!/usr/bin/env python3
"""HBM copy roof on the halo grid's size: torch's copy_ against our dwordx4 grid-stride copy
(copy16_k) and the 7-point stencil at its default tuning, all on the same 512^3 x 3 f64 padded
grid. Rates count one read and one write of every byte moved.

  python scripts/copy_roof.py [--n 512] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, nq, g = a.n, 3, 3
    P = nq * (n + 2 * g + 16)
    G = torch.randn(n + 2 * g, n + 2 * g, P, dtype=torch.float64, device="cuda")
    O = torch.empty_like(G)
    nb = G.numel() * 8
    st = torch.cuda.current_stream().cuda_stream
    us = timed(lambda: O.copy_(G), a.reps)
    print(json.dumps({"what": "torch copy_", "bytes": nb, "us": round(us, 1),
                      "TBps": round(2 * nb / us / 1e6, 2)}), flush=True)
    us = timed(lambda: tz._tz.kernels.copy_bytes(O.data_ptr(), G.data_ptr(), nb, st), a.reps)
    print(json.dumps({"what": "copy16_k", "bytes": nb, "us": round(us, 1),
                      "TBps": round(2 * nb / us / 1e6, 2)}), flush=True)
    x0 = nq * (g + 13)
    row, xs, sy, sz, so, nouter = nq * n, nq, P, P * (n + 2 * g), 0, 1
    base = g * sz + g * sy + x0
    interior = 2 * 8 * n ** 3 * nq
    tz._tz.kernels.set_stencil_tuning()
    us = timed(lambda: tz._tz.kernels.stencil7(G.data_ptr(), O.data_ptr(), base, row, n, n, nouter,
                                               sy, sz, so, xs, 0.4, 0.1, True, st), a.reps)
    print(json.dumps({"what": "stencil7 (lds, default tuning)", "bytes": interior // 2,
                      "us": round(us, 1), "TBps": round(interior / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
