#!/usr/bin/env python3
"""Time the stencil-mode regions on the 512^3 x 3 halo grid: interior [1,n-1)^3, the one-cell
shell, the whole interior.

  python scripts/stencil_regions.py [--order qxyz]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="qxyz")
    ap.add_argument("--n", type=int, default=512)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=a.order, transport="direct",
                                 stencil=True), tz.SelfCtrl(), device=0)
    for region, name in ((0, "interior"), (1, "shell"), (2, "full")):
        ts = []
        for _ in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.stencil(region, st)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"order": a.order, "region": name, "us": round(statistics.median(ts[2:]), 1)}))


if __name__ == "__main__":
    main()
