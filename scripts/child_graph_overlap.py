"""Do parallel branches of a hipGraph overlap? Independent ops on distinct streams compiled into
one hipGraph by the runtime, in one whole-schedule capture (TZ_GRAPH_CAPTURE=schedule, the
default) or as child graphs (TZ_GRAPH_CAPTURE=child; the env is read once per process, so run
this script once per setting).

  python scripts/child_graph_overlap.py [kernels|host]

kernels: two busy kernels (one workgroup each, ~200 us); host: the same plus a host function
(hipLaunchHostFunc, a host node: what RCCL's network proxies add) on a third stream. Prints one
JSON line: per-iteration time, the serial time of one kernel, the graph's node types."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz

    variant = sys.argv[1] if len(sys.argv) > 1 else "kernels"
    us = 200.0
    ops = [tz.BusyKernelOp("a", us), tz.BusyKernelOp("b", us)]
    if variant == "host":
        ops.append(tz.HostFuncOp("h"))
    names = [o.name for o in ops]
    g = tz.Graph()
    for op in ops:
        g.start_then(op)
        g.then_finish(op)
    ns = len(ops)
    seq = None
    for seed in range(400):  # a schedule with every op on a stream of its own
        s = tz.random_rollout(tz.State(g, tz.Platform(ns)), seed)
        st = {o.name: o.stream for o in s.ops() if o.name in names}
        if len(set(st.values())) == ns:
            seq = s
            break
    rt = tz.HipRuntime(device=0, n_streams=ns, mode=tz.ExecMode.Graph)
    rt.prepare(seq)
    rt.run(5)
    rt.device_sync()
    n = 50
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        rt.run(n)
        rt.device_sync()
        dt = (time.perf_counter() - t0) / n
        best = dt if best is None else min(best, dt)
    print(json.dumps({"variant": variant, "capture": os.environ.get("TZ_GRAPH_CAPTURE", "schedule"),
                      "nodes": rt.graph_nodes(), "node_types": rt.graph_node_types(),
                      "mode": str(rt.effective_mode), "iter_us": best * 1e6, "one_kernel_us": us}))


if __name__ == "__main__":
    main()
