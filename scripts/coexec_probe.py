#!/usr/bin/env python3
"""Do the halo move and the SpMV run at the same time on one GPU when nothing joins them?

One torch hipGraph per case, 20 iterations each, replayed 20 times (event-timed, per
iteration):
  move      : 20 x the 26-direction direct move (one stream)
  spmv      : 20 x the local CSR SpMV (m = 150,000, nnz = 10 m)
  serial    : 20 x (move; spmv) on one stream
  coexec    : 20 x move on stream A and 20 x spmv on stream B, one fork and one join per graph
If coexec is close to max(move, spmv), a single kernel holding both (or a schedule without a
per-iteration join) can hide the SpMV under the move; if it is close to serial, they contend.

  python3 scripts/coexec_probe.py [--lanes 1004] [--n 512]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--lanes", default="1004,8", help="SpMV kernels (lanesPerRow codes)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo

    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order="qxyz", transport="direct"),
                      tz.SelfCtrl(), 0)
    dirs = list(range(h.ndirs()))
    m = 150_000
    rp, ci, val = tz._tz.random_band_matrix(m, m, 10 * m, 1)
    rp_t = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci_t = torch.tensor(ci, dtype=torch.int32, device="cuda")
    v_t = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(m, device="cuda")
    y = torch.zeros(m, device="cuda")
    k = tz._tz.kernels

    def move(st):
        h.direct_group(dirs, st.cuda_stream)

    def spmv(st, lanes):
        k.csr_spmv(m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                   y.data_ptr(), lanes, False, st.cuda_stream)

    def timed(build):
        s0 = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s0):
            build(s0)  # warm-up outside the capture
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s0):
            build(s0)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            g.replay()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / (a.reps * a.iters), 2)

    side = torch.cuda.Stream()
    for lanes in (int(v) for v in a.lanes.split(",")):
        def b_move(st):
            for _ in range(a.iters):
                move(st)

        def b_spmv(st):
            for _ in range(a.iters):
                spmv(st, lanes)

        def b_serial(st):
            for _ in range(a.iters):
                move(st)
                spmv(st, lanes)

        def b_coexec(st):
            side.wait_stream(st)
            for _ in range(a.iters):
                move(st)
            with torch.cuda.stream(side):
                for _ in range(a.iters):
                    spmv(side, lanes)
            st.wait_stream(side)

        def b_coexec_spmv_first(st):
            side.wait_stream(st)
            with torch.cuda.stream(side):
                for _ in range(a.iters):
                    spmv(side, lanes)
            for _ in range(a.iters):
                move(st)
            st.wait_stream(side)

        ms = [dict(src=h.grid_ptr(), dst=h.grid_ptr(), src_off=d["src_off"], dst_off=d["dst_off"],
                   len=d["len"], n1=d["n"][0], n2=d["n"][1], n3=d["n"][2], s1=d["s"][0],
                   s2=d["s"][1], s3=d["s"][2], pair=d["pair"]) for d in h.direct_moves(dirs)]
        args = (m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(), y.data_ptr())

        def b_one(st):  # horizontal fusion: both in one launch (ILP kernels only)
            for _ in range(a.iters):
                k.box_move_spmv(ms, *args, lanes if lanes > 1000 else 1004, False, st.cuda_stream)

        r = {"lanes": lanes}
        for name, b in (("move", b_move), ("spmv", b_spmv), ("serial", b_serial),
                        ("coexec", b_coexec), ("coexec_spmv_first", b_coexec_spmv_first),
                        ("one_launch", b_one)):
            r[name + "_us"] = timed(b)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
