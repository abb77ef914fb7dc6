"""Core SDP semantics through the Python API (no GPU). Mirrors the reference's doctest cases
(src/operation.cpp:87-101, src/graph.cpp:422-501, test/test_noop_graph.cpp,
test/test_gpu_graph.cu) and adds synchronizer / serdes / equivalence properties."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def diamond(tz, a=10, b=100, c=100, d=10):
    g = tz.Graph()
    k = {n: tz.SimGpuOp(n, t) for n, t in (("k1", a), ("k2", b), ("k3", c), ("k4", d))}
    g.start_then(k["k1"])
    g.then(k["k1"], k["k2"])
    g.then(k["k1"], k["k3"])
    g.then(k["k2"], k["k4"])
    g.then(k["k3"], k["k4"])
    g.then_finish(k["k4"])
    return g


def normalized(g):
    g2 = g.clone()
    g2.normalize()
    return g2


def test_native_unit_suite():
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-unit")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "0 failures" in r.stderr


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_native_unit_suite_under_sanitizers(kind):
    """the host core (graph, synchronizer, solvers, TCP control plane with ranks as
    threads) under AddressSanitizer + UBSan and under ThreadSanitizer. Any report fails."""
    from tenzing_amd import _build

    exe = _build.build_sanitized(kind)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "0 failures" in r.stderr
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


@pytest.mark.skipif(shutil.which("cmake") is None, reason="no cmake")
def test_cmake_build_of_the_core(tmp_path):
    """the CMake project (for C++ programs that embed the engine, as the reference's drivers link
    its `tenzing` library) configures, builds the host-only core and its unit suite passes"""
    b = tmp_path / "b"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    r = subprocess.run(["cmake", "-S", ROOT, "-B", str(b), *gen, "-DTZ_BUILD_EXAMPLES=OFF"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run(["cmake", "--build", str(b), "--target", "tz-unit", "-j", "8"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run([str(b / "tz-unit")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "0 failures" in r.stderr, r.stderr[-3000:]


def test_noop_graph(tz):
    g = tz.Graph()
    op1 = tz.NoOp("op1")
    g.start_then(op1)
    g.then_finish(op1)
    s = tz.State(g, tz.Platform(2))
    assert len(s.sequence) == 1
    ds = s.get_decisions()
    assert sum(d.kind == "Execute" and d.op.name == "op1" for d in ds) == 1
    for d in ds:
        assert len(s.apply(d).sequence) == 2


def test_graph_api(tz):
    g = diamond(tz)
    g.normalize()
    assert len(g) == 6 and g.num_edges() == 6
    k2 = g.find("k2")
    g2 = g.clone_but_replace(k2, tz.SimGpuOp("k2x", 1))
    assert g2.find("k2x") == k2 and g.find("k2") == k2
    dot = g.dump_graphviz("t")
    assert "digraph" in dot and "k3" in dot
    j = json.loads(g.json())
    assert len(j["vertices"]) == 6
    # erase an edge, then a vertex (reference Graph::erase_edge_only / erase)
    g.erase_edge("k2", "k4")
    assert g.num_edges() == 5 and g.find("k4") not in g.succs(k2)
    g.erase("k3")
    assert len(g) == 5 and not g.contains("k3") and g.num_edges() == 3
    with pytest.raises(Exception, match="no op"):
        g.erase("nope")


def test_op_json_schema(tz):
    """schedule JSON keeps the reference schema"""
    assert json.loads(tz.EventRecord(2, 1, "x").json()) == {
        "name": "x", "stream": 1, "event": 2, "kind": "CudaEventRecord"}
    assert json.loads(tz.StreamWaitEvent(0, 3, "w").json())["kind"] == "CudaStreamWaitEvent"
    assert json.loads(tz.EventSync(3, "s").json()) == {"name": "s", "event": 3, "kind": "CudaEventSync"}
    assert json.loads(tz.NoOp("n").json()) == {"name": "n", "kind": "NoOp"}
    b = tz.BoundGpuOp(tz.SimGpuOp("k", 1), 2)
    assert json.loads(b.json()) == {"name": "k", "stream": 2}


def test_rollouts_are_race_free_and_roundtrip(tz):
    g = diamond(tz)
    ng = normalized(g)
    idx = tz.OpIndex(g)
    for streams in (1, 2, 3, 4):
        for seed in range(30):
            seq = tz.random_rollout(tz.State(g, tz.Platform(streams)), seed)
            assert tz.verify(seq, ng, streams) == []
            back = idx.sequence_from_json(seq.json(True))
            assert back.canonical_key() == seq.canonical_key()
            pruned, k = tz.remove_redundant_syncs(seq, ng, streams)
            assert tz.verify(pruned, ng, streams) == []
            assert len(pruned) == len(seq) - k


def test_verify_catches_missing_sync(tz):
    g = diamond(tz)
    ng = normalized(g)
    ops = {n: ng.op(ng.find(n)) for n in ("k1", "k2", "k3", "k4")}
    s = tz.Sequence()
    s.append(tz.Start())
    s.append(tz.BoundGpuOp(ops["k1"], 0))
    s.append(tz.BoundGpuOp(ops["k2"], 1))
    s.append(tz.BoundGpuOp(ops["k3"], 0))
    s.append(tz.BoundGpuOp(ops["k4"], 0))
    s.append(tz.Finish())
    v = tz.verify(s, ng, 2)
    assert any("k2 not ordered after k1" in x for x in v)
    assert any("Finish" in x for x in v)


def test_stream_symmetry_pruning(tz):
    g = diamond(tz)
    sym = tz.get_all_sequences(g, tz.Platform(3, symmetric_streams=True))
    keys = {s.canonical_key() for s in sym}
    assert len(keys) == len(sym)
    # more streams only add schedules (relabelings of the 3-stream ones are folded)
    sym4 = tz.get_all_sequences(g, tz.Platform(4, symmetric_streams=True))
    assert keys <= {s.canonical_key() for s in sym4}
    # without symmetry folding the raw enumeration is strictly larger
    nosym = tz.get_all_sequences(g, tz.Platform(3, symmetric_streams=False))
    assert len(nosym) >= len(sym)


def test_transitive_host_sync_is_recognized(tz):
    """a -> CES -> b on another stream needs no extra CSWE (vector-clock synchronizer)."""
    g = tz.Graph()
    a, b = tz.SimGpuOp("a", 1), tz.SimGpuOp("b", 1)
    h = tz.NoOp("h")
    g.start_then(a)
    g.then(a, h)
    g.then(a, b)
    g.then(h, b)
    g.then_finish(b)
    s = tz.State(g, tz.Platform(2, symmetric_streams=False))

    def step(pred):
        for d in s.get_decisions():
            if pred(d):
                return s.apply(d)
        raise AssertionError([d.desc() for d in s.get_decisions()])

    s = step(lambda d: d.kind == "Assign" and d.stream == 0)   # a -> s0
    s = step(lambda d: d.kind == "Execute" and d.op.name == "a")
    s = step(lambda d: d.kind == "Execute" and d.op.kind == "CudaEventRecord")
    s = step(lambda d: d.kind == "Execute" and d.op.kind == "CudaEventSync")
    s = step(lambda d: d.kind == "Execute" and d.op.name == "h")
    s = step(lambda d: d.kind == "Assign" and d.stream == 1)   # b -> s1
    names = [d.op.name for d in s.get_decisions() if d.kind == "Execute"]
    assert names == ["b"]  # host already synced with a; no CSWE needed


def test_choice_and_compound(tz):
    sub = tz.Graph()
    x = tz.SimGpuOp("x", 5)
    ch = tz.StaticChoiceOp("y", [tz.SimGpuOp("y_slow", 50), tz.SimGpuOp("y_fast", 5)])
    sub.start_then(x)
    sub.then(x, ch)
    sub.then_finish(ch)
    g = tz.Graph()
    comp = tz.StaticCompoundOp("comp", sub)
    g.start_then(comp)
    g.then_finish(comp)
    s = tz.State(g, tz.Platform(2))
    ds = s.get_decisions()
    assert [d.kind for d in ds] == ["Expand"]
    s = s.apply(ds[0])
    assert s.graph.find("comp") < 0 and s.graph.find("x") > 0
    seqs = tz.get_all_sequences(g, tz.Platform(2))
    names = {op.name for seq in seqs for op in seq.ops()}
    assert {"y_slow", "y_fast"} <= names


def test_equivalence(tz):
    g = diamond(tz)
    s = tz.State(g, tz.Platform(2, symmetric_streams=False))
    ds = [d for d in s.get_decisions() if d.kind == "Assign"]
    assert len(ds) == 2
    a, b = s.apply(ds[0]), s.apply(ds[1])
    # distinguishable streams (priorities / CU masks): bindings are not interchangeable
    assert not a.equivalent(b)
    # ... but the executed sequences are equivalent under a stream bijection (reference
    # get_equivalence(Seq, Seq))
    a = a.apply([d for d in a.get_decisions() if d.kind == "Execute"][0])
    b = b.apply([d for d in b.get_decisions() if d.kind == "Execute"][0])
    assert a.sequence.equivalent(b.sequence)


def test_prime_factors_and_runs_test(tz):
    assert tz._tz.prime_factors(8) == [2, 2, 2]
    assert tz._tz.prime_factors(12) == [3, 2, 2]
    assert tz._tz.runs_test(list(range(40)))
    assert not tz._tz.runs_test([1.0, 2.0, 3.0])
    assert tz._tz.runs_test([1.0, 2.0, 3.0], reject_small=True)


def test_bench_result_percentiles(tz):
    r = tz.BenchResult.from_times([float(i) for i in range(100)])
    assert r.pct01 == 1 and r.pct10 == 10 and r.pct50 == 50 and r.pct99 == 99


def test_graph_then_survives_node_reallocation(tz):
    """start_then/then_finish pass references into the node table; adding the other endpoint
    may grow it (regression: a dangling Start reference became a null op)"""
    g = tz.Graph()
    ops = [tz.SimGpuOp(f"op{i}", 1.0) for i in range(300)]
    for o in ops:
        g.start_then(o)
        g.then_finish(o)
    assert len(g) == 302
    assert g.num_edges() == 600
    for o in ops[:5]:
        assert g.preds(g.find(o.name)) == [0]


def test_xcd_remap_mode_is_validated(tz):
    """only the three block orders exist; a typo must not be recorded as a remap measurement"""
    k = tz._tz.kernels
    prev = k.get_xcd_remap()
    try:
        for m in (0, 1, 2):
            k.set_xcd_remap(m)
            assert k.get_xcd_remap() == m
        for bad in (-1, 3, 17):
            with pytest.raises(ValueError):
                k.set_xcd_remap(bad)
            assert k.get_xcd_remap() == 2
    finally:
        k.set_xcd_remap(prev)


def test_put_block_cap_tunable(tz):
    k = tz._tz.kernels
    prev = k.get_put_max_blocks()
    try:
        k.set_put_max_blocks(128)
        assert k.get_put_max_blocks() == 128
        with pytest.raises(Exception):
            k.set_put_max_blocks(0)
    finally:
        k.set_put_max_blocks(prev)


def test_device_timer_falls_back_to_host_clock(tz):
    """runners without a device clock (host executor) keep the host wall clock"""
    g = tz.Graph()
    a = tz.SleepOp("a", 300.0)
    g.start_then(a)
    g.then_finish(a)
    seq = tz.random_rollout(tz.State(g, tz.Platform(1)), 0)
    b = tz.EmpiricalBenchmarker(tz.HostExecutor(1), tz.SelfCtrl())
    o = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.002, device_timer=True)
    assert o.device_timer
    assert b.benchmark(seq, o).pct10 > 250e-6


def test_racing_cuts_slow_candidates_short(tz):
    """BenchOpts.race_ratio: after the fast alternative has a complete measurement, clearly
    slower candidates stop after race_min measurements; the best one keeps full statistics"""
    g = tz.Graph()
    alts = [tz.SleepOp("fast", 100.0), tz.SleepOp("slow", 900.0), tz.SleepOp("slower", 1500.0)]
    c = tz.StaticChoiceOp("pick", alts)
    g.start_then(c)
    g.then_finish(c)
    b = tz.EmpiricalBenchmarker(tz.HostExecutor(1), tz.SelfCtrl())
    o = tz.DfsOpts()
    o.bench = tz.BenchOpts(n_iters=6, max_retries=1, target_secs=0.002, race_ratio=1.5)
    r = tz.dfs_explore(g, tz.Platform(1), b, tz.SelfCtrl(), o)
    names = [[op.name for op in s.seq.ops()] for s in r.sims]
    t = {next(n for n in ns if n in ("fast", "slow", "slower")): s.res.pct10 for ns, s in zip(names, r.sims)}
    assert t["fast"] < t["slow"] < t["slower"]
    # DFS takes the alternatives in order: fast first, then both slower ones are raced
    assert names[0] == ["Start", "fast", "Finish"] and b.raced == 2


def _nested_choice_graph(tz):
    sub = tz.Graph()
    x = tz.SimGpuOp("x", 5)
    inner = tz.StaticChoiceOp("y", [tz.SimGpuOp("y_slow", 50), tz.SimGpuOp("y_fast", 5)])
    sub.start_then(x)
    sub.then(x, inner)
    sub.then_finish(inner)
    alt_a = tz.StaticCompoundOp("form_a", sub)
    alt_b = tz.SimGpuOp("form_b", 30)
    g = tz.Graph()
    pre = tz.SimGpuOp("pre", 3)
    top = tz.StaticChoiceOp("form", [alt_a, alt_b])
    g.start_then(pre)
    g.then(pre, top)
    g.then_finish(top)
    return g


def test_resolve_graph_verifies_loaded_schedules(tz):
    """a schedule read back from JSON is checked against the graph it executed: choices
    replaced by the alternative it ran, compounds expanded"""
    g = _nested_choice_graph(tz)
    idx = tz.OpIndex(g)
    seen = set()
    for seed in range(40):
        st = tz.State(g, tz.Platform(2))
        seq = tz.random_rollout(st, seed)
        back = idx.sequence_from_json(seq.json(True))
        fg = tz.resolve_graph(g, back)
        names = {fg.op(v).name for v in fg.vertices()}
        assert not {"form", "y", "form_a"} & names  # nothing left to choose or expand
        assert tz.verify(back, fg, 2) == []
        ran = {op.name for op in back.ops()}
        seen.add(frozenset(ran & {"form_b", "y_slow", "y_fast"}))
    assert len(seen) == 3  # every resolution path was exercised
    # an alternative that is not run cannot be resolved
    with pytest.raises(tz.TzError, match="no alternative"):
        tz.resolve_graph(g, tz.Sequence())


def test_resolve_graph_flags_a_dropped_sync(tz):
    g = _nested_choice_graph(tz)
    for seed in range(40):
        seq = tz.random_rollout(tz.State(g, tz.Platform(2, symmetric_streams=False)), seed)
        ops = seq.ops()
        syncs = [i for i, op in enumerate(ops) if op.kind == "CudaStreamWaitEvent"]
        if not syncs:
            continue
        cut = tz.Sequence()
        for i, op in enumerate(ops):
            if i != syncs[0]:
                cut.append(op)
        assert tz.verify(cut, tz.resolve_graph(g, cut), 2) != []
        return
    pytest.skip("no rollout needed a cross-stream wait")


def test_node_identity_is_fixed_size_and_stable(tz):
    """IPC handles travel with this id; a peer maps them only when the ids match (same node)"""
    import socket

    a, b = tz._tz.node_identity(), tz._tz.node_identity()
    assert a == b and len(a) == 96
    assert a.split(b"|")[0] == socket.gethostname().encode()[:63]


def test_settling_stops_consistent_candidates_early(tz):
    """BenchOpts.settle_ratio: once settle_min measurements agree within the ratio, the
    candidate is done (no need for all n_iters); off by default"""
    import time

    g = tz.Graph()
    c = tz.StaticChoiceOp("pick", [tz.SleepOp("a", 100.0), tz.SleepOp("b", 300.0)])
    g.start_then(c)
    g.then_finish(c)
    for settle in (2.0, 0.0):
        b = tz.EmpiricalBenchmarker(tz.HostExecutor(1), tz.SelfCtrl())
        o = tz.DfsOpts()
        o.bench = tz.BenchOpts(n_iters=40, max_retries=1, target_secs=0.002, settle_ratio=settle)
        t0 = time.time()
        r = tz.dfs_explore(g, tz.Platform(1), b, tz.SelfCtrl(), o)
        wall = time.time() - t0
        assert len(r.sims) == 2
        if settle:
            # (a loaded test host can stall one batch past any ratio: at least one settles)
            assert 1 <= b.settled <= 2 and wall < 2.0
        else:
            assert b.settled == 0
    assert tz.BenchOpts(settle_ratio=0.1).settle_ratio == 0.1
