#!/usr/bin/env python3
"""Host-side cost per launch (us) of the halo kernels vs an empty kernel: the eager executor
pays this for every op of every iteration.

  python scripts/launch_cost.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def host_us(fn, n=3000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    torch.zeros(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    K = tz._tz.kernels
    h, _ = build_halo(HaloConfig(n=32, neighbors=26, order="qxyz", transport="direct"),
                      tz.SelfCtrl(), device=0)
    hc, _ = build_halo(HaloConfig(n=32, neighbors=26, order="qxyz", transport="copy"),
                       tz.SelfCtrl(), device=0)
    alld = list(range(h.ndirs()))
    rows = {
        "empty_kernel": host_us(lambda: K.empty(st)),
        "direct_1box": host_us(lambda: h.direct(0, st)),
        "direct_26box": host_us(lambda: h.direct_group(alld, st)),
        "pack_1box": host_us(lambda: hc.pack(0, st)),
        "pack_26box": host_us(lambda: hc.pack_all(st)),
        "copy_26": host_us(lambda: hc.shift_all(st)),
    }
    print(json.dumps({k: round(v, 2) for k, v in rows.items()}), flush=True)


if __name__ == "__main__":
    main()
