"""Isolate hipGraph stream-capture problems: python scripts/diag_capture.py CASE"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402

case = sys.argv[1]
ctrl = tz.SelfCtrl()


def run(g, streams, seed=0):
    rt = tz.HipRuntime(device=0, n_streams=streams, mode=tz.ExecMode.Graph)
    seq = tz.random_rollout(tz.State(g, tz.Platform(streams)), seed)
    print(case, "seq:", seq.desc(), flush=True)
    rt.prepare(seq)
    print(case, "effective", rt.effective_mode, flush=True)
    rt.run(2)
    rt.device_sync()
    print(case, "ok", flush=True)


if case == "empty1":
    g = tz.Graph()
    k = tz.EmptyKernelOp("k")
    g.start_then(k)
    g.then_finish(k)
    run(g, 1)
elif case == "empty2":
    g = tz.Graph()
    a, b, c = tz.EmptyKernelOp("a"), tz.EmptyKernelOp("b"), tz.EmptyKernelOp("c")
    g.start_then(a)
    g.then(a, b)
    g.then(a, c)
    g.then_finish(b)
    g.then_finish(c)
    for seed in range(4):
        run(g, 2, seed)
elif case in ("selfwait", "dupwait", "crosswait"):
    a, b = tz.EmptyKernelOp("a"), tz.EmptyKernelOp("b")
    s = tz.Sequence()
    s.append(tz.Start())
    s.append(tz.BoundGpuOp(a, 0))
    s.append(tz.EventRecord(0, 0))
    if case == "selfwait":
        s.append(tz.StreamWaitEvent(0, 0))
        s.append(tz.BoundGpuOp(b, 0))
    elif case == "dupwait":
        s.append(tz.StreamWaitEvent(1, 0))
        s.append(tz.StreamWaitEvent(1, 0))
        s.append(tz.BoundGpuOp(b, 1))
    else:
        s.append(tz.StreamWaitEvent(1, 0))
        s.append(tz.BoundGpuOp(b, 1))
    s.append(tz.EventRecord(1, 1 if case != "selfwait" else 0))
    s.append(tz.EventSync(1))
    s.append(tz.Finish())
    rt = tz.HipRuntime(device=0, n_streams=2, mode=tz.ExecMode.Graph)
    print(case, s.desc(), flush=True)
    rt.prepare(s)
    rt.run(2)
    rt.device_sync()
    print(case, "ok", flush=True)
elif case.startswith("halo"):
    streams = int(case[4:] or 1)
    h, g = build_halo(HaloConfig(n=24, neighbors=6), ctrl, device=0)
    run(g, streams)
    h.init_grid()
    print("check", h.check_grid())
