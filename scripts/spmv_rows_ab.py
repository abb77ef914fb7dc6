"""Lanes-per-row CSR SpMV with 1, 2 or 4 rows per lane group (loads of several rows in flight)
against the CSR-stream kernel, at the reference's SpMV size (m = 150,000, nnz = 10 m, band width
m: the one-rank case), interleaved rounds of back-to-back launches timed with events.

  python scripts/spmv_rows_ab.py [--m 150000] [--bw 0] [--rounds 5] [--reps 200]
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
    ap.add_argument("--bw", type=int, default=0, help="band width (0: m)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    m, K = a.m, tz._tz.kernels
    rp, ci, val = tz._tz.random_band_matrix(m, a.bw or m, 10 * m, 1)
    rp_t = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci_t = torch.tensor(ci, dtype=torch.int32, device="cuda")
    v_t = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(m, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    variants = [("stream", -1, 1)] + [(f"w{w}_r{r}", w, r) for w in (4, 8, 16) for r in (1, 2, 4)]
    ys = {n: torch.zeros(m, device="cuda") for n, _, _ in variants}
    res = {n: [] for n, _, _ in variants}
    prev = K.get_spmv_rows()
    for _ in range(a.rounds):
        for n, w, r in variants:
            K.set_spmv_rows(r)

            def run():
                K.csr_spmv(m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                           ys[n].data_ptr(), w, False, st)
            for _ in range(5):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    K.set_spmv_rows(prev)
    ref = ys["w8_r1"].double()
    for n, _, _ in variants:
        v = sorted(res[n])
        err = float(((ys[n].double() - ref).abs() / ref.abs().clamp(min=1)).max())
        print(json.dumps({"kernel": n, "median_us": round(v[len(v) // 2], 2), "min_us": round(v[0], 2),
                          "max_rel_diff_vs_w8_r1": err}), flush=True)


if __name__ == "__main__":
    main()
