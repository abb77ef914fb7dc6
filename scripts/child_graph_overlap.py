"""Do parallel branches of a hipGraph overlap? Independent ops on distinct streams compiled into
one hipGraph by the runtime, in one whole-schedule capture (TZ_GRAPH_CAPTURE=schedule, the
default) or as child graphs (TZ_GRAPH_CAPTURE=child; the env is read once per process, so run
this script once per setting).

  python scripts/child_graph_overlap.py [kernels|host|kernel3|hostchain|chainhost]

kernels: two busy kernels (one workgroup each, ~200 us); host: the same plus a host function
(hipLaunchHostFunc, a host node: what RCCL's network proxies add) on a third stream; kernel3: a
third, 50 us kernel instead (control); hostchain / chainhost: a third branch of a host node then
a 50 us kernel (RCCL's shape over its network transport) / the other order. Prints one
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
    chain = []  # (first, second): one branch of two ops in order, on a stream of its own
    if variant == "host":
        ops.append(tz.HostFuncOp("h"))
    elif variant == "kernel3":  # control: a third, short kernel branch
        ops.append(tz.BusyKernelOp("c", 50.0))
    elif variant == "kernel4":  # and a fourth
        ops += [tz.BusyKernelOp("c", 50.0), tz.BusyKernelOp("d", 50.0)]
    elif variant.startswith("equal"):  # equalN: N independent 200 us kernels
        ops = [tz.BusyKernelOp(chr(ord("a") + i), us) for i in range(int(variant[5:]))]
    elif variant.startswith("fork"):  # forkN: N 200 us kernels behind one empty kernel
        ops = [tz.BusyKernelOp(chr(ord("a") + i), us) for i in range(int(variant[4:]))]
    elif variant == "hostchain":  # RCCL's shape: a host node, then a kernel behind it
        chain = [tz.HostFuncOp("h"), tz.BusyKernelOp("c", 50.0)]
    elif variant == "chainhost":  # the other order: a kernel, then a host node
        chain = [tz.BusyKernelOp("c", 50.0), tz.HostFuncOp("h")]
    names = [o.name for o in ops] + ([chain[0].name] if chain else [])
    g = tz.Graph()
    root = tz.EmptyKernelOp("root") if variant.startswith("fork") else None
    if root is not None:
        g.start_then(root)
    for op in ops:
        if root is not None:
            g.then(root, op)
        else:
            g.start_then(op)
        g.then_finish(op)
    if chain:
        g.start_then(chain[0])
        g.then(chain[0], chain[1])
        g.then_finish(chain[1])
    ns = len(names)
    # every branch on a stream of its own, a chain on one stream
    from tenzing_amd.search import greedy_schedule

    sid = {n: i for i, n in enumerate(names)}
    if root is not None:  # the root alone on stream 0, every branch on a stream of its own after it
        sid = {n: i + 1 for i, n in enumerate(names)}
        sid["root"] = 0
        ns += 1
    if chain:
        sid[chain[1].name] = sid[chain[0].name]
    seq = greedy_schedule(g, tz.Platform(ns, symmetric_streams=False), stream_for=lambda n: sid[n])
    eager = os.environ.get("TZ_OVERLAP_EAGER") == "1"
    # TZ_OVERLAP_STREAMS: the runtime owns this many streams (at least the schedule's)
    nrt = max(ns, int(os.environ.get("TZ_OVERLAP_STREAMS", "0")))
    rt = tz.HipRuntime(device=0, n_streams=nrt, mode=tz.ExecMode.Eager if eager else tz.ExecMode.Graph)
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
    print(json.dumps({"variant": variant, "runtime_streams": nrt, "capture": os.environ.get("TZ_GRAPH_CAPTURE", "schedule"),
                      "nodes": rt.graph_nodes(), "node_types": rt.graph_node_types(),
                      "mode": str(rt.effective_mode), "iter_us": best * 1e6, "one_kernel_us": us}))


if __name__ == "__main__":
    main()
