#!/usr/bin/env python3
"""BASELINE config 5 (SpMV + halo in one graph) on one GPU: the time of a few fixed schedules,
eager and as hipGraphs, next to the halo and the SpMV alone -- where does the fused time go?"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused, build_halo, build_spmv
    from tenzing_amd.search import greedy_schedule
    from tenzing_amd.utils.benchkit import timed_replay

    ctrl = tz.SelfCtrl()
    n = int(os.environ.get("N", "512"))
    steps = 50
    out = {}

    def time_seq(rt, seq, label):
        r = {}
        for mode, unroll in ((tz.ExecMode.Eager, 1), (tz.ExecMode.Graph, 20)):
            rt.set_graph_unroll(unroll)
            t, eff = timed_replay(tz, rt, ctrl, seq, mode, steps, 5)
            r[str(mode).split(".")[-1]] = None if t is None else round(t / steps * 1e3, 5)
        r["node_types"] = rt.graph_node_types()
        out[label] = r
        print(label, json.dumps(r), flush=True)

    h, g = build_halo(HaloConfig(n=n, neighbors=26, order="qxyz", fuse="choice"), ctrl, 0)
    rt = tz.HipRuntime(device=0, n_streams=4)
    time_seq(rt, greedy_schedule(g, tz.Platform(4), {"*": ["allfused"]}), "halo_alone")
    del rt, h, g
    s, g = build_spmv(SpmvConfig(m=150_000), ctrl, 0)
    rt = tz.HipRuntime(device=0, n_streams=2)
    for form in ("accum", "split"):
        for k in ("w16", "i4"):
            time_seq(rt, greedy_schedule(g, tz.Platform(2), {"*": [form, k]}), f"spmv_{form}_{k}_s0")
    del rt, s, g
    h, s, g = build_fused(HaloConfig(n=n, neighbors=26, order="qxyz", fuse="choice"), SpmvConfig(m=150_000), ctrl, 0)
    rt = tz.HipRuntime(device=0, n_streams=4)
    kern = os.environ.get("SPMV_KERNEL", "i4")
    pref = {"*": ["allfused", "accum", kern]}
    time_seq(rt, greedy_schedule(g, tz.Platform(4), pref), "fused_all_stream0")
    time_seq(rt, greedy_schedule(g, tz.Platform(4), pref,
                                 stream_for=lambda nm: 1 if nm.startswith("he_") else 0), "fused_halo_s1")
    time_seq(rt, greedy_schedule(g, tz.Platform(4), pref,
                                 stream_for=lambda nm: 1 if nm.startswith("he_") else (2 if "yr" in nm else 0)),
             "fused_halo_s1_yr_s2")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
