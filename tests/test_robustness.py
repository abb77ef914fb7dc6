"""Robustness of the multi-rank search, on the CPU: the RCCL ordering rule, dead-transport
pruning, the host-staged fallback graph, per-transport seed schedules, the control plane's
alltoallv and the run deadline that still reports when a collective hangs.

The reference has no counterpart for most of this: a failed MPI transfer aborted its job, and
its Slurm script's SIGABRT + trap (scripts/perlmutter/spmv.sh:12, src/trap.cpp:26-30) was the
only way a run that could not finish still wrote its partial results.
"""
import json
import os
import random
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- happens-before (independent)

def happens_before_pairs(seq, n_streams):
    """Replay `seq` with vector clocks written here from scratch (not the engine's SyncModel) and
    return a function ordered(i, j): GPU op at position i completes before GPU op j starts."""
    import tenzing_amd as tz

    S = n_streams
    host = [0] * S                 # what the host knows complete, per stream
    stream = [[0] * S for _ in range(S)]  # per stream: what its next op waits for
    count = [0] * S
    events = {}
    stamp = {}                     # position -> (stream, k)
    clock_at = {}                  # position -> clock the op started with
    for pos, op in enumerate(seq.ops()):
        kind = op.kind
        if isinstance(op, tz._tz.BoundGpuOp):
            s = op.stream
            stream[s] = [max(a, b) for a, b in zip(stream[s], host)]
            clock_at[pos] = list(stream[s])
            count[s] += 1
            stamp[pos] = (s, count[s])
            stream[s][s] = count[s]
        elif kind == "CudaEventRecord":
            s = op.stream
            stream[s] = [max(a, b) for a, b in zip(stream[s], host)]
            c = list(stream[s])
            c[s] = count[s]
            events[op.event] = c
        elif kind == "CudaStreamWaitEvent":
            s = op.stream
            stream[s] = [max(a, b) for a, b in zip(stream[s], host)]
            if op.event in events:
                stream[s] = [max(a, b) for a, b in zip(stream[s], events[op.event])]
        elif kind == "CudaEventSync":
            if op.event in events:
                host = [max(a, b) for a, b in zip(host, events[op.event])]
        elif kind == "StreamSync":
            s = op.stream
            c = list(stream[s])
            c[s] = count[s]
            host = [max(a, b) for a, b in zip(host, c)]
        elif kind == "StreamWait":
            raise AssertionError("StreamWait is not offered by default")

    def ordered(i, j):
        s, k = stamp[i]
        return clock_at[j][s] >= k

    return ordered


def rccl_positions(seq):
    return [p for p, op in enumerate(seq.ops()) if op.order_domain == "rccl"]


def _halo(tz, size, transport="auto", fuse="choice", wide_puts="auto", ipc_grid=-1):
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.transport, a.fuse, a.wide_puts = 26, transport, fuse, wide_puts
    a.rank, a.size, a.ipc_grid = 0, size, ipc_grid
    h = tz.HaloExchange(a)
    g = tz.Graph()
    h.add_to_graph(g)
    return h, g


# ---------------------------------------------------------------- ordering rule

def test_rccl_ops_carry_the_domain(tz):
    h, g = _halo(tz, 8, transport="rccl", fuse="none")
    seq = tz.random_rollout(tz.State(g, tz.Platform(4)), 0)
    shifts = [op for op in seq.ops() if op.name.startswith("he_shift_")]
    assert len(shifts) == 26 and all(op.order_domain == "rccl" for op in shifts)
    assert all(op.order_domain == "" for op in seq.ops() if op.name.startswith(("he_pack_", "he_unpack_")))


@pytest.mark.parametrize("fuse", ["none", "pack", "choice"])
@pytest.mark.parametrize("size", [2, 8])
def test_no_two_rccl_ops_unordered_in_random_schedules(tz, fuse, size):
    """every pair of RCCL ops of a schedule is ordered by happens-before (checked by a replay
    independent of the engine), however the search spreads them over 4 streams"""
    h, g = _halo(tz, size, transport="rccl" if fuse != "choice" else "auto", fuse=fuse)
    S = 4
    seen_multi_stream = False
    for seed in range(25):
        seq = tz.random_rollout(tz.State(g, tz.Platform(S)), seed)
        seq, _ = tz.remove_redundant_syncs(seq, tz.resolve_graph(g, seq), S)
        assert tz.verify(seq, tz.resolve_graph(g, seq), S) == []
        pos = rccl_positions(seq)
        ops = seq.ops()
        if len({ops[p].stream for p in pos}) > 1:
            seen_multi_stream = True
        ordered = happens_before_pairs(seq, S)
        for a in range(len(pos)):
            for b in range(a + 1, len(pos)):
                assert ordered(pos[a], pos[b]), (seed, ops[pos[a]].name, ops[pos[b]].name)
    if fuse in ("none", "pack"):
        assert seen_multi_stream  # the rule is exercised, not trivially met on one stream


def test_verify_flags_unordered_domain_ops(tz):
    g = tz.Graph()
    a = tz.SimGpuOp("a", 5, domain="rccl")
    b = tz.SimGpuOp("b", 5, domain="rccl")
    g.start_then(a)
    g.start_then(b)
    g.then_finish(a)
    g.then_finish(b)
    st = tz.State(g, tz.Platform(2))
    # every complete schedule orders a and b (an event edge when they sit on different streams)
    for seed in range(20):
        seq = tz.random_rollout(st, seed)
        ops = seq.ops()
        pa = [i for i, o in enumerate(ops) if o.name == "a"][0]
        pb = [i for i, o in enumerate(ops) if o.name == "b"][0]
        first, second = sorted((pa, pb))
        assert happens_before_pairs(seq, 2)(first, second)
    # a hand-made schedule without the edge is a violation
    bad = tz.Sequence()
    for op in (tz.Start(), tz.BoundGpuOp(a, 0), tz.BoundGpuOp(b, 1), tz.EventRecord(0, 0),
               tz.EventRecord(1, 1), tz.EventSync(0), tz.EventSync(1), tz.Finish()):
        bad.append(op)
    v = tz.verify(bad, g, 2)
    assert v and "b not ordered after a" in v[0]
    # the same ops without a domain are independent: no violation
    g2 = tz.Graph()
    a2, b2 = tz.SimGpuOp("a", 5), tz.SimGpuOp("b", 5)
    for x in (a2, b2):
        g2.start_then(x)
        g2.then_finish(x)
    ok = tz.Sequence()
    for op in (tz.Start(), tz.BoundGpuOp(a2, 0), tz.BoundGpuOp(b2, 1), tz.EventRecord(0, 0),
               tz.EventRecord(1, 1), tz.EventSync(0), tz.EventSync(1), tz.Finish()):
        ok.append(op)
    assert tz.verify(ok, g2, 2) == []


def test_redundant_sync_removal_keeps_domain_edges(tz):
    g = tz.Graph()
    ops = [tz.SimGpuOp(f"c{i}", 5, domain="rccl") for i in range(4)]
    for o in ops:
        g.start_then(o)
        g.then_finish(o)
    for seed in range(20):
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
        red, _ = tz.remove_redundant_syncs(seq, g, 3)
        pos = rccl_positions(red)
        ordered = happens_before_pairs(red, 3)
        assert all(ordered(pos[i], pos[i + 1]) for i in range(len(pos) - 1))


# ---------------------------------------------------------------- dead transports

def _choice_graph(tz, calls, die_on_call=1, die=True):
    """Start -> k0 -> {via_rccl: r (domain rccl) | via_ipc: p} -> k1 -> Finish, plus an
    independent op so the tree has stream choices"""
    def rccl_fn(_stream):
        calls["rccl"] += 1
        if die and calls["rccl"] == die_on_call:
            tz.mark_domain_dead("rccl", "test: simulated watchdog abort")
            raise RuntimeError("RCCL communicator was aborted (test)")

    def ipc_fn(_stream):
        calls["ipc"] += 1

    g = tz.Graph()
    k0, k1, side = tz.SimGpuOp("k0", 5), tz.SimGpuOp("k1", 5), tz.SimGpuOp("side", 20)
    gr = tz.Graph()
    r = tz.PyGpuOp("x_rccl", rccl_fn, 10.0, True, "rccl")
    gr.start_then(r)
    gr.then_finish(r)
    gi = tz.Graph()
    p = tz.PyGpuOp("x_ipc", ipc_fn, 12.0)
    gi.start_then(p)
    gi.then_finish(p)
    ch = tz.StaticChoiceOp("via", [tz.StaticCompoundOp("via_rccl", gr), tz.StaticCompoundOp("via_ipc", gi)])
    g.start_then(k0)
    g.then(k0, ch)
    g.then(ch, k1)
    g.then_finish(k1)
    g.start_then(side)
    g.then_finish(side)
    return g


def test_dead_domain_registry(tz):
    tz.revive_domains()
    assert tz.dead_domains() == []
    tz.mark_domain_dead("rccl", "test")
    assert tz.domain_dead("rccl") and tz.dead_domains() == ["rccl"]
    assert tz.agree_dead_domains(tz.SelfCtrl()) == ["rccl"]
    tz.revive_domains()
    assert not tz.domain_dead("rccl")


def test_mcts_prunes_a_dead_transport(tz):
    tz.revive_domains()
    calls = {"rccl": 0, "ipc": 0}
    g = _choice_graph(tz, calls)
    ex = tz.HostExecutor(2)
    bench = tz.EmpiricalBenchmarker(ex, tz.SelfCtrl())
    opts = tz.MctsOpts()
    opts.n_iters = 60
    opts.bench = tz.BenchOpts(n_iters=2, max_retries=1, target_secs=0.0)
    res = tz.mcts_explore(g, tz.Platform(2), bench, tz.SelfCtrl(), opts)
    try:
        assert calls["rccl"] == 1           # measured once (and died), never again
        assert res.failed == 1
        assert res.dead_domains == ["rccl"]
        assert res.pruned_dead >= 1
        assert calls["ipc"] > 0 and res.sims
        for s in res.sims:
            assert not any(o.name == "x_rccl" for o in s.seq.ops())
    finally:
        tz.revive_domains()


def test_dfs_skips_sequences_of_a_dead_transport(tz):
    tz.revive_domains()
    calls = {"rccl": 0, "ipc": 0}
    g = _choice_graph(tz, calls)
    bench = tz.EmpiricalBenchmarker(tz.HostExecutor(2), tz.SelfCtrl())
    opts = tz.DfsOpts()
    opts.bench = tz.BenchOpts(n_iters=2, max_retries=1, target_secs=0.0)
    res = tz.dfs_explore(g, tz.Platform(2), bench, tz.SelfCtrl(), opts)
    try:
        assert calls["rccl"] == 1
        assert res.dead_domains == ["rccl"] and res.pruned_dead > 0
        assert all(not any(o.name == "x_rccl" for o in s.seq.ops()) for s in res.sims)
    finally:
        tz.revive_domains()


def test_every_alternative_dead_stops_the_search(tz):
    tz.revive_domains()
    tz.mark_domain_dead("rccl", "test")
    g = tz.Graph()
    r = tz.SimGpuOp("only_rccl", 5, domain="rccl")
    g.start_then(r)
    g.then_finish(r)
    try:
        bench = tz.SimBenchmarker(1, tz.SimParams())
        opts = tz.MctsOpts()
        opts.n_iters = 20
        res = tz.mcts_explore(g, tz.Platform(1), bench, tz.SelfCtrl(), opts)
        assert res.sims == [] and res.stop_reason == "full_tree"
    finally:
        tz.revive_domains()


# ---------------------------------------------------------------- host-staged transport graph

@pytest.mark.parametrize("size", [2, 8])
def test_host_transport_graph(tz, size):
    h, g = _halo(tz, size, transport="host")
    assert h.uses_host() and "host" in h.transport() and not h.uses_rccl()
    for seed in range(6):
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
        names = [o.name for o in seq.ops()]
        assert not any(n.startswith("he_shift_") for n in names)
        i, x, u = (names.index(n) for n in ("he_pack_host", "he_hostxfer", "he_unpack_host"))
        assert i < x < u
        # the host op follows the pack's completion (an event sync before it)
        assert any(o.kind == "CudaEventSync" for o in seq.ops()[i:x])
        assert tz.verify(seq, tz.resolve_graph(g, seq), 3) == []
    if size == 2:
        assert h.uses_direct()


# ---------------------------------------------------------------- seeds

def test_one_seed_per_transport(tz, monkeypatch):
    """buffers mode, 8 ranks (2x2x2): one schedule per he_remote alternative, each using its
    transport; measured as seeds, every one lands in the tree"""
    from tenzing_amd.search import choice_alternatives, greedy_schedule

    h, g = _halo(tz, 8, wide_puts="on", ipc_grid=0)
    alts = choice_alternatives(g, "he_remote")
    assert {"he_via_rccl", "he_via_ipc", "he_via_ipcw", "he_via_sdma", "he_via_memcpy",
            "he_via_mixed"} <= set(alts)
    assert any(a.startswith("he_via_relay") for a in alts)
    p = tz.Platform(4)
    key = {"he_via_rccl": "he_shift_", "he_via_ipc": "he_put_", "he_via_ipcw": "he_putw_",
           "he_via_sdma": "he_copyput_",
           "he_via_memcpy": "he_mcput_", "he_via_mixed": "he_wait_mx", "he_via_hs10": "he_hs10", "he_via_hs20": "he_hs20",
           "he_via_hs30": "he_hs30", "he_via_hs40": "he_hs40"}
    seeds = []
    for alt in alts:
        s = greedy_schedule(g, p, {"he_remote": alt, "*": ["allfused", "fused"]})
        names = [o.name for o in s.ops()]
        want = key.get(alt, "he_rl")
        assert any(n.startswith(want) for n in names), (alt, names)
        assert tz.verify(s, tz.resolve_graph(g, s), 4) == []
        seeds.append(s)
    opts = tz.MctsOpts()
    opts.n_iters = 5
    opts.seed_schedules = seeds
    res = tz.mcts_explore(g, p, tz.SimBenchmarker(4, tz.SimParams()), tz.SelfCtrl(), opts)
    assert sum(s.seeded for s in res.sims) == len(seeds)
    assert res.counter_counts().get("SEED_IN_TREE", 0) == len(seeds)


# ---------------------------------------------------------------- multi-process

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(body, world, tmp_path, timeout=120, env=None):
    """run `body` (source of a function `main(c) -> dict` with c the control plane) on `world`
    ranks; returns [(returncode, stdout, stderr)] per rank"""
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {ROOT!r})
        import tenzing_amd as tz
        from tenzing_amd.parallel import init_ctrl
        {textwrap.indent(textwrap.dedent(body), '        ').strip()}
        c = init_ctrl(timeout_s=60)
        r = main(c)
        if r is not None:
            print("RESULT " + json.dumps(r), flush=True)
    """))
    port = _free_port()
    procs = []
    for rank in range(world):
        e = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TZ_LOG="warn")
        e.update(env or {})
        procs.append(subprocess.Popen([sys.executable, str(script)], env=e, cwd=str(tmp_path),
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    out = []
    for p in procs:
        try:
            o, er = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            o, er = p.communicate()
        out.append((p.returncode, o, er))
    return out


def _result(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("RESULT ")]
    return json.loads(lines[-1][7:]) if lines else None


def test_alltoallv_two_and_three_ranks(tmp_path):
    body = """
    def main(c):
        out = [bytes([c.rank * 16 + j]) * (1000 * (c.rank + 1) + j) for j in range(c.size)]
        got = c.alltoallv(out)
        return {"lens": [len(x) for x in got], "first": [x[0] for x in got]}
    """
    for world in (2, 3):
        res = _spawn(body, world, tmp_path)
        for rank, (rc, o, e) in enumerate(res):
            assert rc == 0, e
            r = _result(o)
            assert r["lens"] == [1000 * (i + 1) + rank for i in range(world)]
            assert r["first"] == [i * 16 + rank for i in range(world)]


def test_simulated_rccl_abort_on_one_rank_prunes_on_all(tmp_path):
    """rank 1's RCCL op dies (a watchdog abort there); the ranks agree, and no rank measures an
    RCCL candidate again"""
    body = """
    calls = {"rccl": 0, "ipc": 0, "recovered": 0}

    def main(c):
        def recover(ctrl):
            calls["recovered"] += 1
            ctrl.barrier()  # hooks may be collective

        tz._tz.add_recovery_hook(recover)

        def rccl_fn(_s):
            calls["rccl"] += 1
            if c.rank == 1 and calls["rccl"] == 1:
                tz._tz.note_abort()
                tz.mark_domain_dead("rccl", "simulated watchdog abort")
                raise RuntimeError("RCCL communicator was aborted (simulated)")

        def ipc_fn(_s):
            calls["ipc"] += 1

        g = tz.Graph()
        k0, side = tz.SimGpuOp("k0", 5), tz.SimGpuOp("side", 20)
        gr, gi = tz.Graph(), tz.Graph()
        r = tz.PyGpuOp("x_rccl", rccl_fn, 10.0, True, "rccl")
        gr.start_then(r); gr.then_finish(r)
        p = tz.PyGpuOp("x_ipc", ipc_fn, 12.0)
        gi.start_then(p); gi.then_finish(p)
        ch = tz.StaticChoiceOp("via", [tz.StaticCompoundOp("via_rccl", gr),
                                       tz.StaticCompoundOp("via_ipc", gi)])
        g.start_then(k0); g.then(k0, ch); g.then_finish(ch)
        g.start_then(side); g.then_finish(side)
        bench = tz.EmpiricalBenchmarker(tz.HostExecutor(2), c)
        opts = tz.MctsOpts()
        opts.n_iters = 40
        opts.bench = tz.BenchOpts(n_iters=2, max_retries=1, target_secs=0.0)
        res = tz.mcts_explore(g, tz.Platform(2), bench, c, opts)
        rccl_measured = sum(any(o.name == "x_rccl" for o in s.seq.ops()) for s in res.sims)
        return {"calls": calls, "dead": list(res.dead_domains), "failed": res.failed,
                "sims": len(res.sims), "rccl_measured": rccl_measured,
                "pruned": res.pruned_dead}
    """
    res = _spawn(body, 2, tmp_path)
    rs = []
    for rc, o, e in res:
        assert rc == 0, e
        rs.append(_result(o))
    for r in rs:
        assert r["dead"] == ["rccl"]
        # the first RCCL candidate ran (on rank 0 completely, on rank 1 until it died); no other
        assert r["calls"]["rccl"] <= 2 * 1 and r["calls"]["ipc"] > 0
        # one rank aborted a run: every rank reset its transports once
        assert r["calls"]["recovered"] == 1
    assert rs[0]["failed"] == 1 and rs[0]["rccl_measured"] == 0 and rs[0]["sims"] > 0
    assert rs[0]["pruned"] >= 1


def test_run_deadline_reports_when_a_collective_hangs(tmp_path):
    """rank 1 never joins the barrier: rank 0 hangs inside a native collective, and its run
    deadline prints the report line (the best result so far, marked partial) and exits 5"""
    body = """
    import time

    def main(c):
        d = tz.RunDeadline(3.0, 5)
        if c.rank == 0:
            d.set_report(json.dumps({"metric": "m", "value": 0.123, "partial": True,
                                     "phase": "search"}))
        if c.rank == 1:
            time.sleep(8)      # never reaches the barrier in time
            d.cancel()
            return None
        c.barrier()            # rank 0 blocks here (GIL released, native wait)
        return {"unreachable": True}
    """
    res = _spawn(body, 2, tmp_path, timeout=60)
    rc0, o0, e0 = res[0]
    assert rc0 == 5, (rc0, o0, e0)
    line = [ln for ln in o0.splitlines() if ln.startswith("{")][-1]
    j = json.loads(line)
    assert j["partial"] is True and j["value"] == 0.123
    assert "run deadline" in e0


def test_fatal_exit_prints_the_partial_report():
    """the watchdog's last resort (a hung run its abort could not release) leaves through
    exit_with_report: the armed deadline's line is printed once, with the reason added, and the
    process exits with the given status (not the deadline's)"""
    import subprocess
    import sys

    code = ("import json, tenzing_amd as tz\n"
            "d = tz.RunDeadline(30.0, 5)\n"
            "d.set_report(json.dumps({'metric': 'm', 'value': 0.5, 'partial': True}))\n"
            "tz._tz.exit_with_report(3, 'watchdog: a \"hung\" run')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 3, (r.stdout, r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["partial"] is True and j["value"] == 0.5
    assert j["exit_reason"] == 'watchdog: a "hung" run'
    assert "partial result printed" in r.stderr


def test_run_deadline_cancel(tz):
    d = tz.RunDeadline(0.5, 5)
    assert d.armed and 0 < d.remaining <= 0.5
    d.cancel()
    import time
    time.sleep(0.8)  # the process is still alive
    assert not d.armed


def test_seed_results_checkpoint_and_callback_indices(tz, tmp_path):
    """seeds keep their flag through a checkpoint and resume, and the result callback's indices
    are the results' positions (seeds first, then the search, no collisions)"""
    from tenzing_amd.search import greedy_schedule

    g = tz.Graph()
    k = [tz.SimGpuOp(f"k{i}", 10 * (i + 1)) for i in range(3)]
    for op in k:
        g.start_then(op)
        g.then_finish(op)
    p = tz.Platform(2)
    seed = greedy_schedule(g, p)
    ck = tmp_path / "ck.json"
    opts = tz.MctsOpts()
    opts.n_iters = 6
    opts.seed_schedules = [seed]
    opts.checkpoint_path = str(ck)
    idx = []
    res = tz.mcts_explore(g, p, tz.SimBenchmarker(2, tz.SimParams()), tz.SelfCtrl(), opts,
                          lambda i, sr: idx.append(i))
    assert idx == list(range(len(res.sims)))
    assert res.sims[0].seeded and not any(s.seeded for s in res.sims[1:])
    doc = json.loads(ck.read_text())
    assert doc["sims"][0].get("seeded") is True
    opts2 = tz.MctsOpts()
    opts2.n_iters = 2
    opts2.resume_path = str(ck)
    res2 = tz.mcts_explore(g, p, tz.SimBenchmarker(2, tz.SimParams()), tz.SelfCtrl(), opts2)
    assert res2.sims[0].seeded
