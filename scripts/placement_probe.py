#!/usr/bin/env python3
"""Where the reference layout's move time comes from: K grids of one layout
allocated side by side in one process (so they sit on different device memory), the
26-direction move of each event-timed, then (under rocprofv3 --pmc) each grid's move run
`--reps` times in grid order, so the per-dispatch counters line up with the timed grids.

  python3 scripts/placement_probe.py --grids 6 [--layout xyzq:-1:0] [--reps 5]
  rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum --output-format csv -d out -o run -- \\
      python3 scripts/placement_probe.py --grids 6 --reps 5
  python3 scripts/placement_probe.py --dispatches out/run_counter_collection.csv --grids 6 --reps 5

One JSON line per grid: its virtual address and move time (the last form: the counter of each
grid's dispatches instead).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dispatches(path, grids, reps):
    """per grid: median counter values of its `reps` move dispatches (file order = issue order)"""
    import csv
    import statistics
    from collections import defaultdict

    rows = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
    order = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "box_move_many_k" not in r["Kernel_Name"]:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(order))
            if d not in rows:
                order.append(d)
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
    order.sort()
    # the timing phase ran 3 + 2 x iters moves per grid first: the profiled reps are the tail
    tail = order[-grids * reps:]
    for g in range(grids):
        ds = tail[g * reps:(g + 1) * reps]
        names = sorted({c for d in ds for c in rows[d]})
        print(json.dumps({"grid": g, **{c: statistics.median(rows[d][c] for d in ds) for c in names}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", type=int, default=6)
    ap.add_argument("--layout", default="xyzq:-1:0", help="order:ghost_align[:pitch_pad]")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5, help="moves per grid for the counters")
    ap.add_argument("--spacer-mb", default="0",
                    help="hold this much device memory before each grid (other placements); a "
                         "comma list gives one size per grid")
    ap.add_argument("--xcd-remaps", default="0",
                    help="comma list of the move's block orders to time per grid (0, 1, 2)")
    ap.add_argument("--dispatches", default="", help="summarize a counter CSV instead")
    a = ap.parse_args()
    if a.dispatches:
        dispatches(a.dispatches, a.grids, a.reps)
        return
    import torch

    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo
    from roof_probe import _time_move

    order, align, *pad = a.layout.split(":")
    pad = int(pad[0]) if pad else 0
    sp = [int(v) for v in a.spacer_mb.split(",")]
    sp = (sp * a.grids)[:a.grids]
    halos, spacers = [], []
    for g in range(a.grids):
        if sp[g] > 0:
            spacers.append(torch.empty(sp[g] << 20, dtype=torch.uint8, device="cuda"))
        h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=order, ghost_align=int(align),
                                     transport="direct", pitch_pad=pad), tz.SelfCtrl(), 0)
        halos.append(h)
    k = tz._tz.kernels
    prev = k.get_xcd_remap()
    for g, h in enumerate(halos):
        va = h.grid_ptr()
        rec = {"grid": g, "layout": a.layout, "spacer_mb": sp[g], "grid_va": hex(va),
               "grid_va_mod_1GB_MB": (va % (1 << 30)) >> 20}
        for mode in (int(v) for v in a.xcd_remaps.split(",")):
            k.set_xcd_remap(mode)
            us = [_time_move(h, a.iters) for _ in range(2)]
            rec["move_us" if mode == 0 else f"move_us_remap{mode}"] = us
        k.set_xcd_remap(prev)
        print(json.dumps(rec), flush=True)
    st = torch.cuda.current_stream().cuda_stream
    for h in halos:
        for _ in range(a.reps):
            h.direct_group(list(range(h.ndirs())), st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
