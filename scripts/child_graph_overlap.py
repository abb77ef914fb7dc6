"""Do parallel branches of a hipGraph still overlap when its nodes are child graphs?

Two independent busy kernels (one workgroup each, ~200 us) on two streams, compiled into a
hipGraph by the runtime in one whole-schedule capture (TZ_GRAPH_CAPTURE=schedule, the default) or
as child graphs (TZ_GRAPH_CAPTURE=child; the env is read once per process, so run this script once
per setting). Prints one JSON line: per-iteration time and the serial time of one kernel."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz

    us = 200.0
    a, b = tz.BusyKernelOp("a", us), tz.BusyKernelOp("b", us)
    g = tz.Graph()
    for op in (a, b):
        g.start_then(op)
        g.then_finish(op)
    seq = None
    for seed in range(100):  # a schedule with a and b on different streams
        s = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
        st = {o.name: o.stream for o in s.ops() if o.name in ("a", "b")}
        if len(set(st.values())) == 2:
            seq = s
            break
    rt = tz.HipRuntime(device=0, n_streams=2, mode=tz.ExecMode.Graph)
    rt.prepare(seq)
    rt.run(5)
    rt.device_sync()
    n = 50
    t0 = time.perf_counter()
    rt.run(n)
    rt.device_sync()
    dt = (time.perf_counter() - t0) / n
    print(json.dumps({"capture": os.environ.get("TZ_GRAPH_CAPTURE", "schedule"), "nodes": rt.graph_nodes(), "mode": str(rt.effective_mode),
                      "iter_us": dt * 1e6, "one_kernel_us": us}))


if __name__ == "__main__":
    main()
