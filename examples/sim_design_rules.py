#!/usr/bin/env python3
"""Hardware-free walk through the engine: build an op graph, enumerate every race-free schedule
with DFS on the discrete-event simulator, then mine the results for design rules
(reference postprocess/postprocess.py).

  python examples/sim_design_rules.py [--out /tmp/rules_]
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tenzing_amd as tz  # noqa: E402
from tenzing_amd.utils import postprocess  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(tempfile.gettempdir(), "tz_example_"))
    a = ap.parse_args()
    # a -> {b, c} -> d: b and c are long and independent; overlapping them is what matters
    g = tz.Graph()
    k = {n: tz.SimGpuOp(n, us) for n, us in (("a", 20), ("b", 100), ("c", 100), ("d", 20))}
    g.start_then(k["a"])
    g.then(k["a"], k["b"])
    g.then(k["a"], k["c"])
    g.then(k["b"], k["d"])
    g.then(k["c"], k["d"])
    g.then_finish(k["d"])
    print(g.dump_graphviz("example"))
    ctrl = tz.SelfCtrl()
    o = tz.DfsOpts()
    o.bench = tz.BenchOpts(n_iters=5)
    res = tz.dfs_explore(g, tz.Platform(2), tz.SimBenchmarker(2), ctrl, o)
    csv = a.out + "results.csv"
    with open(csv, "w") as f:
        f.write(res.dump_csv())
    best = res.sims[res.best()]
    print(f"{len(res.sims)} schedules; best pct10 {best.res.pct10 * 1e6:.1f} us:")
    print(best.seq.desc())
    return postprocess.main([csv, "--out", a.out])


if __name__ == "__main__":
    sys.exit(main())
