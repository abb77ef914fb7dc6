"""What one search candidate costs before its first measurement: `HipRuntime.prepare` (event
provisioning; in graph mode the capture of 1 and of `--unroll` iterations into hipGraphs,
instantiation and upload) for random schedules of the headline halo graph.

  python scripts/prepare_cost.py [--unroll 10] [--seqs 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unroll", type=int, default=10)
    ap.add_argument("--seqs", type=int, default=20)
    ap.add_argument("--streams", type=int, default=4)
    a = ap.parse_args()
    h, g = build_halo(HaloConfig(n=512, neighbors=26, order="qxyz", fuse="choice"),
                      tz.SelfCtrl(), device=0)
    seqs = [tz.random_rollout(tz.State(g, tz.Platform(a.streams)), s) for s in range(a.seqs)]
    for mode, unroll in (("eager", 1), ("graph", 1), ("graph", a.unroll)):
        rt = tz.HipRuntime(device=0, n_streams=a.streams,
                           mode=tz.ExecMode.Graph if mode == "graph" else tz.ExecMode.Eager,
                           graph_unroll=unroll)
        ts, runs = [], []
        for seq in seqs:
            t0 = time.perf_counter()
            rt.prepare(seq)
            ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            rt.run(unroll)
            rt.device_sync()
            runs.append(time.perf_counter() - t0)
        print(json.dumps({"mode": mode, "unroll": unroll,
                          "prepare_ms_median": round(statistics.median(ts) * 1e3, 3),
                          "prepare_ms_max": round(max(ts) * 1e3, 3),
                          "ops_median": statistics.median(len(s) for s in seqs),
                          "first_run_ms_median": round(statistics.median(runs) * 1e3, 3)}))
        del rt
    return 0


if __name__ == "__main__":
    sys.exit(main())
