#!/usr/bin/env python3
"""Isolated CSR SpMV kernel timings (MI355X): every lanes-per-row variant, the CSR-stream
kernel and the rocSPARSE CSR algorithms (library comparison) on the SpMV workload's local block
(m=150,000, nnz=10 m by default).

  python scripts/spmv_bench.py [--m 150000] [--reps 200]
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
    ap.add_argument("--m", type=int, default=150_000)
    ap.add_argument("--per-row", type=int, default=10)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--bw", type=int, default=0, help="band half-width (0: m, as at one rank)")
    a = ap.parse_args()
    rp, ci, val = tz._tz.random_band_matrix(a.m, a.bw or a.m, a.per_row * a.m, 1)
    dev = "cuda"
    rp_t = torch.tensor(rp, dtype=torch.int32, device=dev)
    ci_t = torch.tensor(ci, dtype=torch.int32, device=dev)
    v_t = torch.tensor(val, dtype=torch.float32, device=dev)
    x = torch.randn(a.m, dtype=torch.float32, device=dev)
    y = torch.zeros(a.m, dtype=torch.float32, device=dev)
    nbytes = rp_t.numel() * 4 + ci_t.numel() * 8 + a.m * 8
    st = torch.cuda.current_stream().cuda_stream
    K = tz._tz.kernels
    variants = [(f"lanes{w}", w) for w in (4, 8, 16, 32)] + [("stream", -1)]
    variants += [(f"ilp{w}", 1000 + w) for w in (1, 2, 4)]
    variants += [(f"rocsparse_{alg}", alg) for alg in ("adaptive", "lrb", "rowsplit")]
    yref = None
    for name, v in variants:
        if isinstance(v, int):
            def fn(lanes=v):
                K.csr_spmv(a.m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                           y.data_ptr(), lanes, False, st)
        else:
            lib = K.RocsparseCsr(a.m, a.m, ci_t.numel(), rp_t.data_ptr(), ci_t.data_ptr(),
                                 v_t.data_ptr(), x.data_ptr(), y.data_ptr(), v)

            def fn(lib=lib):
                lib.run(st)
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        if yref is None:
            yref = y.clone()
        err = float((y - yref).abs().max() / yref.abs().max().clamp_min(1e-30))
        print(json.dumps({"variant": name, "us": round(us, 2), "nnz": ci_t.numel(),
                          "GBps": round(nbytes / us / 1e3, 1), "rel_err_vs_lanes4": err}),
              flush=True)


if __name__ == "__main__":
    main()
