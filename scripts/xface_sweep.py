#!/usr/bin/env python3
"""Direct-move x-face throughput vs row-pitch padding (QXYZ): the x faces are 72-byte runs one
row pitch apart, so the pitch decides how those runs spread over HBM channels.

  python scripts/xface_sweep.py [--pads 0,16,32,64,128,256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pads", default="0,16,32,48,64,128,256")
    ap.add_argument("--order", default="qxyz")
    ap.add_argument("--n", type=int, default=512)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for pad in [int(p) for p in a.pads.split(",")]:
        h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=a.order, transport="direct",
                                     pitch_pad=pad), tz.SelfCtrl(), device=0)
        xf = [i for i in range(h.ndirs()) if h.dir(i) in ((1, 0, 0), (-1, 0, 0))]
        allv = list(range(h.ndirs()))
        xb = sum(h.box_elems(i) for i in xf) * 16
        r = {"pad": pad, "pitch": h.pack_box(xf[0])["s1"],
             "xfaces_us": round(timeit(lambda: h.direct_group(xf, st), 50), 2),
             "all_us": round(timeit(lambda: h.direct_group(allv, st), 50), 2)}
        r["xfaces_GBps"] = round(xb / r["xfaces_us"] / 1e3, 1)
        print(json.dumps(r), flush=True)
        del h
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
