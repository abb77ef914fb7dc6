#!/usr/bin/env python3
"""7-point stencil kernel on the halo workload's 512^3 x 3 f64 grid: LDS-tiled vs direct, both
storage orders; effective HBM rate = (interior bytes read + written) / time.

  python scripts/stencil_bench.py [--n 512] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--orders", default="qxyz,xyzq")
    ap.add_argument("--zcs", default="32,64", help="z-chunk lengths to sweep (16, 32, 64)")
    ap.add_argument("--pfs", default="1,2")
    ap.add_argument("--dbs", default="1,0")
    ap.add_argument("--xcds", default="0", help="tile orders: 0 hardware, 1 XCD-contiguous")
    ap.add_argument("--rounds", type=int, default=1,
                    help="time every configuration this many times, interleaved (one line each)")
    ap.add_argument("--no-direct", action="store_true", help="skip the non-LDS kernel")
    a = ap.parse_args()
    n, nq, g = a.n, 3, 3
    st = torch.cuda.current_stream().cuda_stream
    for order in a.orders.split(","):
        if order == "qxyz":
            P = nq * (n + 2 * g + 16)
            G = torch.randn(n + 2 * g, n + 2 * g, P, dtype=torch.float64, device="cuda")
            x0 = nq * (g + 13)
            row, xs, sy, sz, so, nouter = nq * n, nq, P, P * (n + 2 * g), 0, 1
        else:
            P = n + 2 * g + 16
            G = torch.randn(nq, n + 2 * g, n + 2 * g, P, dtype=torch.float64, device="cuda")
            x0 = g + 13
            row, xs, sy, sz, nouter = n, 1, P, P * (n + 2 * g), nq
            so = sz * (n + 2 * g)
        O = torch.empty_like(G)
        base = g * sz + g * sy + x0
        nbytes = 2 * 8 * n ** 3 * nq
        configs = [(True, ty, int(zc), int(pf), db == "1", x == "1") for ty in (8, 16)
                   for zc in a.zcs.split(",") for pf in a.pfs.split(",") for db in a.dbs.split(",")
                   for x in a.xcds.split(",")]
        if not a.no_direct:
            configs += [(False, 8, 32, 1, False, False)]
        configs = configs * max(1, a.rounds)
        # roof: torch's contiguous copy of the whole padded grid (read + write every element)
        for _ in range(3):
            O.copy_(G)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            O.copy_(G)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        us = statistics.median(ts)
        print(json.dumps({"order": order, "copy_roof": True, "us": round(us, 1),
                          "TBps": round(2 * 8 * G.numel() / us / 1e6, 2)}), flush=True)
        for lds, ty, zc, pf, db, xcd in configs:
            tz._tz.kernels.set_stencil_tuning(ty, zc, pf, db)
            tz._tz.kernels.set_stencil_xcd_tiles(xcd)

            def fn():
                tz._tz.kernels.stencil7(G.data_ptr(), O.data_ptr(), base, row, n, n, nouter, sy, sz,
                                        so, xs, 0.4, 0.1, lds, st)
            for _ in range(3):
                fn()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = statistics.median(ts)
            print(json.dumps({"order": order, "lds": lds, "ty": ty, "zc": zc, "pf": pf, "db": db,
                              "xcd_tiles": xcd, "us": round(us, 1),
                              "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
        del G, O
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
