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


def _time_move(halo, iters):
    """us per 26-direction move, event-timed over `iters` back-to-back launches after 3 warm-up"""
    import torch

    st = torch.cuda.current_stream()
    dirs = list(range(halo.ndirs()))
    for _ in range(3):
        halo.direct_group(dirs, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        halo.direct_group(dirs, st.cuda_stream)
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


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
    ap.add_argument("--prealloc-mb", default="0",
                    help="comma list: before each layout's grid is allocated, hold this many MB "
                         "of device memory, so the grid lands on other physical memory (one "
                         "JSON line per layout and size)")
    a = ap.parse_args()
    import torch

    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo

    specs = [(spec, int(mb)) for mb in a.prealloc_mb.split(",") for spec in a.layouts.split(",")]
    for spec, mb in specs:
        hold = torch.empty(mb << 20, dtype=torch.uint8, device="cuda") if mb > 0 else None
        order, align, *pad = spec.split(":")
        pad = int(pad[0]) if pad else 0
        halo, _ = build_halo(HaloConfig(n=a.n, neighbors=a.neighbors, order=order,
                                        ghost_align=int(align), transport="direct",
                                        move_pairs=a.pairs == "on", pitch_pad=pad),
                             tz.SelfCtrl(), 0)
        try:
            r = halo.move_roof(a.iters)
            r["move_over_roof"] = min(r["move_us"], r["move_us_again"]) / r["roof_us"]
        except RuntimeError as e:
            # no line-shaped roof for this layout (row strides not whole 128-B lines): the move
            # alone, event-timed, back to back on one stream
            r = {"roof": str(e), "move_us": _time_move(halo, a.iters),
                 "move_us_again": _time_move(halo, a.iters)}
        va = halo.grid_ptr()
        r.update(order=order, ghost_align=int(align), pitch_pad=pad, layout=halo.layout(),
                 move_pairs=a.pairs, prealloc_mb=mb, grid_va=hex(va),
                 grid_va_mod_2MB=va % (2 << 20), grid_va_mod_1GB=va % (1 << 30))
        print(json.dumps(r), flush=True)
        del halo, hold
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
