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
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order="qxyz", transport="direct"),
                      tz.SelfCtrl(), device=0)
    k = tz._tz.kernels
    st = torch.cuda.current_stream()
    dirs = list(range(h.ndirs()))
    unroll, ntp, ntu, mb, ntm = k.get_box_tuning()
    # name: (nt loads, nt stores, unroll, xcd remap, max blocks per box)
    variants = {"r1_default": (True, False, 4, 0, 4096), "nt_both": (True, True, 4, 0, 4096),
                "plain": (False, False, 4, 0, 4096), "default": (False, True, 4, 0, 4096)}
    if a.extra:
        variants.update({"default_u8": (False, True, 8, 0, 4096),
                         "default_remap1": (False, True, 4, 1, 4096),
                         "default_remap2": (False, True, 4, 2, 4096),
                         "default_mb1024": (False, True, 4, 0, 1024),
                         "default_mb16384": (False, True, 4, 0, 16384)})
    res = {v: [] for v in variants}
    prev_remap = k.get_xcd_remap()
    for r in range(a.rounds):
        for name, (ntload, ntstore, u, remap, mbv) in variants.items():
            k.set_box_tuning(u, ntp, ntu, mbv, ntload)
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


if __name__ == "__main__":
    main()
