"""Bounded failure on the GPU: the watchdog's floor + k x expected deadline with the device abort
flag, and the RCCL preflight (passing, and a hang that is cut off instead of blocking setup).
Multi-rank fallbacks (IPC refused -> host-staged transport) are in test_gpu_multirank.py."""
import time

import pytest

pytestmark = pytest.mark.gpu


def _hang_graph(tz, hang_s=1000.0):
    """Start -> {slow: a kernel that spins for `hang_s` | fast: an empty kernel} -> Finish"""
    g = tz.Graph()
    slow, fast = tz.Graph(), tz.Graph()
    h = tz.BusyKernelOp("hang", hang_s * 1e6, 1)
    e = tz.EmptyKernelOp("quick")
    slow.start_then(h)
    slow.then_finish(h)
    fast.start_then(e)
    fast.then_finish(e)
    ch = tz.StaticChoiceOp("which", [tz.StaticCompoundOp("slow", slow), tz.StaticCompoundOp("fast", fast)])
    g.start_then(ch)
    g.then_finish(ch)
    return g


def _schedule(tz, g, want):
    from tenzing_amd.search import greedy_schedule

    return greedy_schedule(g, tz.Platform(2), {"which": want})


def test_watchdog_aborts_a_hung_ten_iteration_graph_batch(tz, gpu):
    g = _hang_graph(tz)
    rt = tz.HipRuntime(device=gpu, n_streams=2, mode=tz.ExecMode.Graph, watchdog_s=5.0,
                       watchdog_k=50.0, graph_unroll=10)
    hang, quick = _schedule(tz, g, "slow"), _schedule(tz, g, "fast")
    rt.prepare(hang)
    assert rt.effective_mode == tz.ExecMode.Graph and rt.expected_iter_s == 0
    assert rt.watchdog_budget(10) == pytest.approx(5.0)  # nothing known yet: the floor alone
    t0 = time.time()
    with pytest.raises(Exception, match="watchdog"):
        rt.run(10)  # one launch of the 10-iteration graph
    took = time.time() - t0
    assert took < 30, took
    assert rt.watchdog_fired == 1 and not tz._tz.device_abort_set()
    # the runtime is usable afterwards, and a schedule that ran once gets floor + k x expected
    rt.prepare(quick)
    rt.run(10)
    rt.device_sync()
    assert rt.expected_iter_s > 0
    assert rt.watchdog_budget(100) == pytest.approx(5.0 + 50.0 * rt.expected_iter_s * 100)
    tz.revive_domains()


def test_search_continues_past_a_hung_candidate(tz, gpu):
    g = _hang_graph(tz)
    rt = tz.HipRuntime(device=gpu, n_streams=2, mode=tz.ExecMode.Graph, watchdog_s=4.0,
                       graph_unroll=10)
    ctrl = tz.SelfCtrl()
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    opts = tz.MctsOpts()
    opts.n_iters = 6
    opts.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
    t0 = time.time()
    res = tz.mcts_explore(g, tz.Platform(2), bench, ctrl, opts)
    took = time.time() - t0
    try:
        assert res.failed == 1 and rt.watchdog_fired == 1, (res.failed, rt.watchdog_fired)
        assert res.sims and all(any(o.name == "quick" for o in s.seq.ops()) for s in res.sims)
        assert took < 40, took
    finally:
        tz.revive_domains()


def test_rccl_preflight_one_rank(tz, gpu):
    """forced RCCL on one rank: every direction goes through RCCL (self send/recv), and setup
    runs the verified per-direction and fused-hipGraph preflight exchanges first"""
    from tenzing_amd.models import HaloConfig, build_halo

    h, g = build_halo(HaloConfig(n=32, neighbors=26, transport="rccl", fuse="choice"),
                      tz.SelfCtrl(), device=gpu)
    rep = h.transport_report()
    # RCCL passed eager and hipGraph preflights, in whole-schedule capture
    assert rep["rccl"] == "ok (hipGraph: schedule capture)" and h.rccl_nranks() == 1, rep
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 0)
    rt = tz.HipRuntime(device=gpu, n_streams=2)
    h.init_grid()
    rt.prepare(seq)
    rt.run(1)
    rt.device_sync()
    assert h.check_grid() == 0


def test_rccl_graph_preflight_falls_back_to_child_capture(tz, gpu, monkeypatch):
    """whole-schedule capture failing the RCCL graph preflight (simulated wrong data) is not the
    end of RCCL in hipGraphs: the preflight moves on to child-graph capture, which passes, and
    the report says which mode RCCL schedules are built in and why"""
    from tenzing_amd.models import HaloConfig, build_halo

    monkeypatch.setenv("TZ_FAIL_TRANSPORTS", "rccl_graph_schedule")
    h, g = build_halo(HaloConfig(n=32, neighbors=6, transport="rccl"), tz.SelfCtrl(), device=gpu)
    rep = h.transport_report()["rccl"]
    assert rep.startswith("ok (hipGraph: child capture (schedule capture: ") and "wrong cells" in rep, rep
    assert h.rccl_graph_ok()
    rt = tz.HipRuntime(device=gpu, n_streams=2, mode=tz.ExecMode.Graph)
    h.init_grid()
    rt.prepare(tz.random_rollout(tz.State(g, tz.Platform(2)), 1))
    assert rt.effective_mode == tz.ExecMode.Graph
    rt.run(2)
    rt.device_sync()
    assert h.check_grid() == 0


def test_rccl_preflight_hang_is_bounded(tz, gpu, monkeypatch):
    """a preflight exchange that never completes (simulated: a spinning kernel ahead of it) is
    cut off after TZ_PREFLIGHT_S: the communicators are aborted and a forced RCCL transport
    fails setup with the reason instead of hanging"""
    from tenzing_amd.models import HaloConfig, build_halo

    monkeypatch.setenv("TZ_FAIL_TRANSPORTS", "rccl_hang")
    monkeypatch.setenv("TZ_PREFLIGHT_S", "3")
    t0 = time.time()
    with pytest.raises(Exception, match="preflight"):
        build_halo(HaloConfig(n=32, neighbors=26, transport="rccl"), tz.SelfCtrl(), device=gpu)
    assert time.time() - t0 < 30
    assert not tz._tz.device_abort_set()


def test_rccl_init_with_a_missing_rank_is_bounded(gpu):
    """a communicator of 2 ranks that only one process joins: the init would block forever; it
    raises after TZ_RCCL_INIT_S instead (the caller then drops RCCL collectively). In a child
    process: the abandoned init thread stays blocked inside RCCL until that process exits."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r); import tenzing_amd as tz; "
            "t0 = time.time()\n"
            "try:\n"
            "    tz._tz.RcclComm.from_id(tz._tz.rccl_unique_id(), 0, 2, %d)\n"
            "    print('JOINED')\n"
            "except Exception as e:\n"
            "    print('RAISED', round(time.time() - t0, 1), e)\n"
            # the abandoned init thread is still inside RCCL: leave without teardown
            "import os; sys.stdout.flush(); os._exit(0)\n" % (root, gpu))
    env = dict(os.environ, TZ_RCCL_INIT_S="4")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90,
                       env=env)
    line = [x for x in r.stdout.splitlines() if x.startswith(("RAISED", "JOINED"))][-1]
    assert line.startswith("RAISED") and "did not complete" in line, (r.stdout, r.stderr[-2000:])
    assert float(line.split()[1]) < 20
