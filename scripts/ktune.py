"""Tune the halo box kernels in pipeline context (pack_all -> shift_all -> unpack_all repeated,
so caches are in the state a real exchange leaves them), interleaving configurations in one
process (methodology: A/B in one process, several rounds, report min/median).

python scripts/ktune.py [--order qxyz] [--rounds 5] [--iters 50]
"""
import argparse
import itertools
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
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--unrolls", default="",
                    help="comma list: sweep items per lane (grid sizing) at the default nt "
                         "settings instead of the round-1 grid (1-2: more workgroups, one item "
                         "in flight; the direct move gained 1.2 %% that way, profiles/archive/r2_move_shape/)")
    a = ap.parse_args()
    torch.zeros(1, device="cuda")
    h, _ = build_halo(HaloConfig(n=a.n, neighbors=26, order=a.order, transport="copy"),
                      tz.SelfCtrl(), device=0)
    s = torch.cuda.current_stream()
    st = s.cuda_stream
    K = tz._tz.kernels
    # (unroll, nt_pack, nt_unpack, max_blocks); first round (r1) showed unroll 8 and block caps
    # neutral, nt pack loads -27 %, nt unpack stores +5 %
    prev = K.get_box_tuning()
    configs = list(itertools.product([4, 8], [False, True], [False, True], [4096]))
    if a.unrolls:
        configs = [(int(u), ntp, ntu, 65535) for u in a.unrolls.split(",") for ntp in (False, True)
                   for ntu in (False, True)]
    res = {c: {"pack": [], "shift": [], "unpack": [], "iter": []} for c in configs}
    for _ in range(a.rounds):
        for c in configs:
            K.set_box_tuning(*c)
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(a.iters)]
            for _ in range(3):
                h.pack_all(st); h.shift_all(st); h.unpack_all(st)
            for i in range(a.iters):
                e = ev[i]
                e[0].record(s); h.pack_all(st)
                e[1].record(s); h.shift_all(st)
                e[2].record(s); h.unpack_all(st)
                e[3].record(s)
            torch.cuda.synchronize()
            pk = [e[0].elapsed_time(e[1]) * 1e3 for e in ev]
            sh = [e[1].elapsed_time(e[2]) * 1e3 for e in ev]
            up = [e[2].elapsed_time(e[3]) * 1e3 for e in ev]
            res[c]["pack"].append(statistics.median(pk))
            res[c]["shift"].append(statistics.median(sh))
            res[c]["unpack"].append(statistics.median(up))
            res[c]["iter"].append(statistics.median([p + q + r for p, q, r in zip(pk, sh, up)]))
    for c in configs:
        r = res[c]
        print(json.dumps({"unroll": c[0], "nt_pack": c[1], "nt_unpack": c[2], "max_blocks": c[3],
                          **{k: round(statistics.median(v), 2) for k, v in r.items()},
                          "iter_min": round(min(r["iter"]), 2)}), flush=True)
    K.set_box_tuning(*prev)


if __name__ == "__main__":
    main()
