#!/usr/bin/env python3
"""The fused direct move of the 26-direction halo against its shape-matched roof, per layout.

Each layout: `HaloExchange.move_roof` times the move and a kernel that touches exactly the same
128-B lines (whole-line 16-B accesses, trivial indexing), back to back on one stream. One JSON
line per layout. Under `rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace` the counters of
both kernels (box_move_many_k, line_roof_k) come out per dispatch.

  python3 scripts/roof_probe.py [--n 512] [--iters 20] [--layouts qxyz:16,xyzq:-1,xyzq:16]
  python3 scripts/roof_probe.py --layouts xyzq:-1:0,xyzq:-1:8,xyzq:-1:16,xyzq:-1:32   # pitch sweep
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--neighbors", type=int, default=26)
    ap.add_argument("--layouts", default="qxyz:16,xyzq:-1,xyzq:16",
                    help="order:ghost_align[:pitch_pad] (-1: x = 0 at the row start, the reference; "
                         "pitch_pad: extra row-pitch elements, 528 + pad for 512^3 XYZQ)")
    ap.add_argument("--pairs", default="on", choices=["on", "off"],
                    help="XYZQ x self-wrap moves as row pairs (HaloConfig.move_pairs)")
    a = ap.parse_args()
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo

    for spec in a.layouts.split(","):
        order, align, *pad = spec.split(":")
        pad = int(pad[0]) if pad else 0
        halo, _ = build_halo(HaloConfig(n=a.n, neighbors=a.neighbors, order=order,
                                        ghost_align=int(align), transport="direct",
                                        move_pairs=a.pairs == "on", pitch_pad=pad),
                             tz.SelfCtrl(), 0)
        r = halo.move_roof(a.iters)
        r.update(order=order, ghost_align=int(align), pitch_pad=pad, layout=halo.layout(),
                 move_pairs=a.pairs)
        r["move_over_roof"] = min(r["move_us"], r["move_us_again"]) / r["roof_us"]
        print(json.dumps(r), flush=True)
        del halo


if __name__ == "__main__":
    main()
