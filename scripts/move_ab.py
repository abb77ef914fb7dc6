"""In-process A/B of the fused 26-direction move kernel (the 1-GPU headline's only kernel):
non-temporal ghost stores on/off (and source loads), interleaved, back-to-back launches like the
hipGraph replay, at the bench's 512^3 x 3 QXYZ geometry.

  python scripts/move_ab.py [--reps 200] [--rounds 5]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--extra", action="store_true", help="also unroll / XCD order / block caps")
    ap.add_argument("--blocks", action="store_true",
                    help="also 1-2 items in flight per lane (2-4x the workgroups; the HBM probe, "
                         "scripts/hbm_roof.hip, copies fastest with ~128 workgroups per CU)")
    ap.add_argument("--groups", action="store_true",
                    help="instead: the default move of each direction group alone (x / y / z "
                         "faces, edges, corners) and all together, with its line traffic rate")
    ap.add_argument("--order", default="qxyz")
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    if a.groups:
        return groups(a)
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order="qxyz", transport="direct"),
                      tz.SelfCtrl(), device=0)
    k = tz._tz.kernels
    st = torch.cuda.current_stream()
    dirs = list(range(h.ndirs()))
    unroll, ntp, ntu, mb, ntm = k.get_box_tuning()
    mu0, mi0 = k.get_move_unroll(), k.get_move_items()
    # name: (nt loads, nt stores, items in flight per lane, XCD remap, max blocks per box
    #        [, items per lane the grid is sized for; default = in flight])
    variants = {"r1_default": (True, False, 4, 0, 4096), "nt_both": (True, True, 4, 0, 4096),
                "plain": (False, False, 4, 0, 4096), "u4": (False, True, 4, 0, 4096)}
    if a.extra:
        variants.update({"u4_remap1": (False, True, 4, 1, 4096),
                         "u4_remap2": (False, True, 4, 2, 4096),
                         "u4_mb1024": (False, True, 4, 0, 1024),
                         "u4_mb16384": (False, True, 4, 0, 16384)})
    if a.blocks:
        # fewer items per lane: 2x / 4x the workgroups for the same boxes
        variants.update({"u2": (False, True, 2, 0, 65535),
                         "u1": (False, True, 1, 0, 65535),
                         "u2_mb4096": (False, True, 2, 0, 4096),
                         "u2_remap1": (False, True, 2, 1, 65535),
                         "u1_remap1": (False, True, 1, 1, 65535),
                         "u2_plain": (False, False, 2, 0, 65535),
                         "u2_nt_both": (True, True, 2, 0, 65535),
                         "u1_i2": (False, True, 1, 0, 65535, 2),
                         "u1_i3": (False, True, 1, 0, 65535, 3),
                         "u2_i4": (False, True, 2, 0, 65535, 4),
                         "u2_i6": (False, True, 2, 0, 65535, 6),
                         "u4_i8": (False, True, 4, 0, 65535, 8)})
    res = {v: [] for v in variants}
    prev_remap = k.get_xcd_remap()
    for r in range(a.rounds):
        for name, (ntload, ntstore, u, remap, mbv, *items) in variants.items():
            k.set_box_tuning(unroll, ntp, ntu, mbv, ntload)
            k.set_move_unroll(u)
            k.set_move_items(items[0] if items else u)
            k.set_nt_move_store(ntstore)
            k.set_xcd_remap(remap)
            for _ in range(5):
                h.direct_group(dirs, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                h.direct_group(dirs, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    k.set_box_tuning(unroll, ntp, ntu, mb, ntm)
    k.set_move_unroll(mu0)
    k.set_move_items(mi0)
    k.set_nt_move_store(True)
    k.set_xcd_remap(prev_remap)
    h.init_grid()
    h.direct_group(dirs, st.cuda_stream)
    torch.cuda.synchronize()
    bad = h.check_grid()
    for name, v in res.items():
        v = sorted(v)
        print(json.dumps({"variant": name, "median_us": round(v[len(v) // 2], 2),
                          "min_us": round(v[0], 2), "all": [round(x, 2) for x in v]}))
    print(json.dumps({"bad_cells_after_default": int(bad)}))


def _lines(moves):
    """128-B lines read + written by these moves (every row at one intra-line alignment)"""
    tot = 0
    for m in moves:
        rows = m["n"][0] * m["n"][1] * m["n"][2]
        runs = [(m["src_off"], m["len"]), (m["dst_off"], m["len"])]
        if m["pair"]:
            d = m["dst_off"] - m["src_off"]
            runs += [(m["src_off"] + m["len"] + d, m["len"]), (m["src_off"] + m["len"], m["len"])]
        for off, ln in runs:
            tot += rows * ((off + ln - 1) // 16 - off // 16 + 1)
    return tot * 128


def groups(a):
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=a.order, transport="direct"),
                      tz.SelfCtrl(), device=0)
    st = torch.cuda.current_stream()
    kind = {}
    for i in range(h.ndirs()):
        d = h.dir(i)
        nz = sum(1 for c in d if c)
        key = ("x", "y", "z")[[c != 0 for c in d].index(True)] + "_faces" if nz == 1 else \
            ("edges" if nz == 2 else "corners")
        kind.setdefault(key, []).append(i)
    kind["all"] = list(range(h.ndirs()))
    for name, dirs in kind.items():
        v = []
        for _ in range(a.rounds):
            for _ in range(3):
                h.direct_group(dirs, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                h.direct_group(dirs, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            v.append(e0.elapsed_time(e1) * 1e3 / a.reps)
        v.sort()
        lines = _lines(h.direct_moves(dirs))
        us = v[len(v) // 2]
        print(json.dumps({"group": name, "dirs": len(dirs), "median_us": round(us, 2),
                          "line_MB": round(lines / 1e6, 2), "TBps": round(lines / us / 1e6, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
