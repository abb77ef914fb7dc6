#!/usr/bin/env python3
"""BASELINE config 5 on one GPU: can the SpMV run beside the halo move if the move leaves
workgroup slots free? The move's workgroups per box are capped (kernels.set_box_tuning
max_blocks; grid-stride beyond), and three schedules are timed as hipGraphs (20 unrolled
iterations) at each cap: the move alone, SpMV after the move on one stream, and the move on
stream 1 beside the SpMV on stream 0.

  python3 scripts/fused_occupancy.py [--caps 4096,1024,512,256,128] [--n 512]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="4096,1024,512,256,192,128")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--kernel", default="i4", help="SpMV local kernel alternative (name part)")
    a = ap.parse_args()
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused
    from tenzing_amd.search import greedy_schedule
    from tenzing_amd.utils.benchkit import timed_replay

    ctrl = tz.SelfCtrl()
    h, s, g = build_fused(HaloConfig(n=a.n, neighbors=26, order="qxyz", fuse="choice"),
                          SpmvConfig(m=150_000), ctrl, 0)
    rt = tz.HipRuntime(device=0, n_streams=4, mode=tz.ExecMode.Graph, graph_unroll=20)
    plat = tz.Platform(4, symmetric_streams=False)
    pref = {"*": ["allfused", "accum", a.kernel]}
    seqs = {
        "serial_s0": greedy_schedule(g, plat, pref),
        "halo_s1_beside_spmv_s0": greedy_schedule(
            g, plat, pref, stream_for=lambda nm: 1 if nm.startswith("he_") else 0),
    }
    k = tz._tz.kernels
    prev = k.get_box_tuning()
    try:
        for cap in (int(c) for c in a.caps.split(",")):
            k.set_box_tuning(prev[0], prev[1], prev[2], cap, prev[4])
            r = {"cap": cap}
            dirs = list(range(h.ndirs()))
            import torch

            st = torch.cuda.current_stream()
            for _ in range(3):
                h.direct_group(dirs, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(50):
                h.direct_group(dirs, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            r["move_alone_us"] = round(e0.elapsed_time(e1) * 1e3 / 50, 2)
            for name, seq in seqs.items():
                t, eff = timed_replay(tz, rt, ctrl, seq, tz.ExecMode.Graph, a.steps, 10)
                r[name + "_us"] = None if t is None else round(t / a.steps * 1e6, 2)
            s.reset_y()
            rt.device_sync()
            rt.set_mode(tz.ExecMode.Eager)
            rt.prepare(seqs["halo_s1_beside_spmv_s0"])
            rt.run(1)
            rt.device_sync()
            r["spmv_err"] = s.check()
            r["halo_bad"] = int(h.check_grid())
            print(json.dumps(r), flush=True)
    finally:
        k.set_box_tuning(*prev)


if __name__ == "__main__":
    main()
