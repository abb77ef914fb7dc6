"""LDS column-panel CSR SpMV against the other local-SpMV variants at the reference's SpMV size
(m = 150,000, nnz = 10 m, band width m: every row gathers across the whole x), back-to-back
launches timed with events, interleaved rounds.

  python scripts/spmv_panel_bench.py [--m 150000] [--rounds 5] [--reps 200]
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
    ap.add_argument("--bw", type=int, default=0, help="band width (0: m, the 1-rank case)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    m = a.m
    K = tz._tz.kernels
    rp, ci, val = tz._tz.random_band_matrix(m, a.bw or m, 10 * m, 1)
    dev = torch.device("cuda")
    rp_t = torch.tensor(rp, dtype=torch.int32, device=dev)
    ci_t = torch.tensor(ci, dtype=torch.int32, device=dev)
    v_t = torch.tensor(val, dtype=torch.float32, device=dev)
    npan, prp, pcol, pval = K.build_panel_csr(rp, ci, val, m, K.PANEL_WIDTH)
    prp_t = torch.tensor(prp, dtype=torch.int32, device=dev)
    pcol_t = torch.tensor(pcol, dtype=torch.int32).to(torch.int16).to(dev)
    pval_t = torch.tensor(pval, dtype=torch.float32, device=dev)
    x = torch.randn(m, device=dev)
    ys = {}
    st = torch.cuda.current_stream().cuda_stream

    def run(name, y):
        if name == "panel":
            K.csr_spmv_panel(m, m, npan, K.PANEL_WIDTH, prp_t.data_ptr(), pcol_t.data_ptr(),
                             pval_t.data_ptr(), x.data_ptr(), y.data_ptr(), False, st)
        else:
            lanes = {"w4": 4, "w8": 8, "w16": 16, "stream": -1}[name]
            K.csr_spmv(m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                       y.data_ptr(), lanes, False, st)

    names = ["w8", "stream", "panel", "w4", "w16"]
    res = {n: [] for n in names}
    for n in names:
        ys[n] = torch.zeros(m, device=dev)
    for _ in range(a.rounds):
        for n in names:
            for _ in range(5):
                run(n, ys[n])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run(n, ys[n])
            e1.record()
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    ref = ys["w8"].double()
    for n in names:
        v = sorted(res[n])
        err = float(((ys[n].double() - ref).abs() / ref.abs().clamp(min=1)).max())
        print(json.dumps({"kernel": n, "median_us": round(v[len(v) // 2], 2), "min_us": round(v[0], 2),
                          "panels": npan if n == "panel" else None, "max_rel_diff_vs_w8": err}),
              flush=True)


if __name__ == "__main__":
    main()
