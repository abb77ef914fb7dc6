"""In-process A/B of the order of the 26 boxes inside the fused move launch (the 1-GPU
headline's only kernel). Blocks are dispatched box by box in batch order; with ~8,800 blocks and
~2,000 resident at a time, the order decides which boxes make up the last waves. The x faces
(strided 72-B runs) cost the most per block, so running them first may shorten the tail.

  python scripts/box_order_ab.py [--reps 200] [--rounds 7]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--n", type=int, default=512)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order="qxyz", transport="direct"),
                      tz.SelfCtrl(), device=0)
    st = torch.cuda.current_stream()
    dirs = list(range(h.ndirs()))
    kind = {i: sum(1 for c in h.dir(i) if c) for i in dirs}  # dir(i) = (dx, dy, dz)
    xface = [i for i in dirs if kind[i] == 1 and h.dir(i)[0] != 0]
    faces = [i for i in dirs if kind[i] == 1]
    rest = [i for i in dirs if kind[i] > 1]
    orders = {
        "natural": dirs,
        "x_faces_first": xface + [i for i in dirs if i not in xface],
        "x_faces_last": [i for i in dirs if i not in xface] + xface,
        "faces_first": faces + rest,
        "small_first": rest + faces,
        "reversed": dirs[::-1],
    }
    res = {k: [] for k in orders}
    for _ in range(a.rounds):
        for name, order in orders.items():
            for _ in range(5):
                h.direct_group(order, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                h.direct_group(order, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    bad = 0
    for order in orders.values():
        h.init_grid()
        h.direct_group(order, st.cuda_stream)
        torch.cuda.synchronize()
        bad += h.check_grid()
    for name, v in res.items():
        v = sorted(v)
        print(json.dumps({"order": name, "median_us": round(v[len(v) // 2], 2),
                          "min_us": round(v[0], 2), "all": [round(x, 2) for x in v]}))
    print(json.dumps({"bad_cells": int(bad)}))


if __name__ == "__main__":
    main()
