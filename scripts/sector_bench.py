#!/usr/bin/env python3
"""A/B of aligned x ghost runs with whole-sector (8) / whole-line (16) direct-move writes
(HaloArgs.ghost_align) against the line-optimal padding (0): the whole 26-direction move and the two x faces alone,
interleaved in one process, several rounds, every configuration verified on the device.

  python scripts/sector_bench.py [--order qxyz] [--rounds 5] [--iters 50]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    halos = {}
    for sg in (0, 8, 16):
        h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=a.order, transport="direct",
                                     ghost_align=sg), tz.SelfCtrl(), device=0)
        h.init_grid()
        h.direct_group(list(range(h.ndirs())), st)
        torch.cuda.synchronize()
        assert h.check_grid() == 0, f"ghost_align={sg}: wrong cells"
        halos[sg] = h
    res = {}
    for _ in range(a.rounds):
        for sg, h in halos.items():
            alld = list(range(h.ndirs()))
            xs = [i for i in alld if h.dir(i) in ((1, 0, 0), (-1, 0, 0))]
            for gname, dirs in (("all26", alld), ("xfaces", xs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(5):
                    h.direct_group(dirs, st)
                e0.record()
                for _ in range(a.iters):
                    h.direct_group(dirs, st)
                e1.record()
                e1.synchronize()
                res.setdefault((gname, sg), []).append(e0.elapsed_time(e1) * 1e3 / a.iters)
    for (gname, sg), v in sorted(res.items()):
        print(json.dumps({"order": a.order, "group": gname, "ghost_align": sg,
                          "us_median": round(statistics.median(v), 2), "us_min": round(min(v), 2)}))


if __name__ == "__main__":
    main()
