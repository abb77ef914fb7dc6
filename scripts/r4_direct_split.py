"""The 1-GPU headline's two structures, timed as the bench times them (hipGraph, 20 iterations
per launch): all 26 directions in one move kernel, or the faces group and the edges+corners
group as two moves, on one stream (serial) or on two streams (concurrent)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.search import greedy_schedule

    halo, g = build_halo(HaloConfig(n=512, neighbors=26, order="qxyz", fuse="choice"),
                         tz.SelfCtrl(), device=0)
    plat = tz.Platform(4, symmetric_streams=False)
    cases = {
        "allfused": ({"he_remote": None, "*": ["allfused"]}, lambda n: 0),
        "groups_serial": ({"*": ["grouped", "fused"]}, lambda n: 0),
        "groups_concurrent": ({"*": ["grouped", "fused"]}, lambda n: 1 if "small" in n else 0),
    }
    rt = tz.HipRuntime(device=0, n_streams=4, mode=tz.ExecMode.Graph, graph_unroll=20)
    for name, (prefer, sf) in cases.items():
        prefer = {k: v for k, v in prefer.items() if v is not None}
        seq = greedy_schedule(g, plat, prefer, stream_for=sf)
        halo.init_grid()
        rt.prepare(seq)
        rt.run(40)
        rt.device_sync()
        best = None
        for _ in range(5):
            t0 = time.perf_counter()
            rt.run(200)
            rt.device_sync()
            dt = (time.perf_counter() - t0) / 200
            best = dt if best is None else min(best, dt)
        bad = halo.check_grid()
        print(json.dumps({"case": name, "us_per_iter": best * 1e6, "bad": int(bad),
                          "ops": [o.name for o in seq.ops() if o.name.startswith("he_")],
                          "streams": sorted({o.stream for o in seq.ops() if o.name.startswith("he_")}),
                          "node_types": rt.graph_node_types()}), flush=True)


if __name__ == "__main__":
    main()
