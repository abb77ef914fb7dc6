"""BASELINE config 5's graph (SpMV + halo) with horizontal fusion: on one rank a top-level
ChoiceOp offers one kernel launch for the 26-direction move and the SpMV's local product
(``hs_onelaunch_i4`` / ``_i2``) beside the two workloads' own ops (``hs_separate``). Graph-only
(no GPU)."""
import pytest

from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused
from tenzing_amd.search import choice_alternatives, greedy_schedule


def _fused(tz, ctrl=None, **kw):
    return build_fused(HaloConfig(n=32, neighbors=26, order="qxyz", fuse="choice", **kw),
                       SpmvConfig(m=3000), ctrl, -1, setup=False)


def test_one_rank_offers_one_launch_for_both_workloads(tz):
    h, s, g = _fused(tz)
    assert choice_alternatives(g, "hs_launches") == ["hs_separate", "hs_onelaunch_i4", "hs_onelaunch_i2"]
    plat = tz.Platform(4)
    one = greedy_schedule(g, plat, {"hs_launches": "hs_onelaunch_i4"})
    names = [o.name for o in one.ops() if isinstance(o, tz._tz.BoundGpuOp)]
    assert names == ["hs_onelaunch_i4"], names
    op = [o for o in one.ops() if isinstance(o, tz._tz.BoundGpuOp)][0].unbound
    assert op.kind == "MoveSpmv" and op.traffic()[0][0] == "hbm"
    sep = greedy_schedule(g, plat, {"hs_launches": "hs_separate", "*": ["allfused", "accum"]})
    sn = [o.name for o in sep.ops() if isinstance(o, tz._tz.BoundGpuOp)]
    assert any(n.startswith("he_direct") for n in sn) and any(n.startswith("spmv_") for n in sn), sn
    # random rollouts reach both structures; every schedule is race-free
    seen = set()
    for seed in range(40):
        seq = tz.random_rollout(tz.State(g, plat), seed)
        gpu = [o.name for o in seq.ops() if isinstance(o, tz._tz.BoundGpuOp)]
        seen.add("one" if any(n.startswith("hs_onelaunch") for n in gpu) else "sep")
        assert tz.verify(seq, tz.resolve_graph(g, seq), 4) == []
    assert seen == {"one", "sep"}
    # the simulator prices the one launch below the two workloads back to back
    p = tz.SimParams()
    t1 = tz.SimExecutor(4, p).run_once(one)
    t2 = tz.SimExecutor(4, p).run_once(greedy_schedule(g, tz.Platform(1), {"hs_launches": "hs_separate",
                                                                            "*": ["allfused", "accum"]}))
    assert t1 < t2


def test_no_one_launch_without_the_precondition(tz):
    # the stencil belongs to the halo graph, so no single launch can replace it
    _, _, g = _fused(tz, stencil=True)
    assert choice_alternatives(g, "hs_launches") == []
    # several ranks: remote directions and remote SpMV parts stay separate ops
    a = build_fused(HaloConfig(n=32, neighbors=26, order="qxyz", fuse="choice"), SpmvConfig(m=3000),
                    None, -1, setup=False, horizontal=False)[2]
    assert choice_alternatives(a, "hs_launches") == []


def test_move_spmv_op_checks_its_arguments(tz):
    h, s, _ = _fused(tz)
    with pytest.raises(Exception, match="lanes"):
        tz._tz.move_spmv_op(h, list(range(h.ndirs())), s, "x", 1003, True)
    with pytest.raises(Exception, match="at most"):
        tz._tz.move_spmv_op(h, list(range(h.ndirs())) * 2, s, "x", 1004, True)


def test_native_cli_builds_the_same_choice(tmp_path):
    """tz-search builds config 5 with the same top-level choice (a schedule saved by either CLI
    names the same ops), and not with --horizontal off"""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tenzing_amd",
                       "bin", "tz-search")
    for hz, want in (("on", True), ("off", False)):
        dot = tmp_path / f"g_{hz}.dot"
        r = subprocess.run([exe, "--workload", "halo+spmv", "--sim", "--iters", "2", "--halo-n", "32",
                            "--neighbors", "26", "--order", "qxyz", "--fuse", "choice", "--spmv-m", "3000",
                            "--horizontal", hz, "--dump-graph", str(dot)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert ("hs_launches" in dot.read_text()) == want
