"""One-call schedule search for a user graph.

``tz.search(graph, ...)`` wires up what every driver otherwise assembles by hand: the control
plane (this process alone, or every rank under ``torchrun``), the HIP runtime or a hardware-free
benchmarker, the benchmark options and the solver. The reference's drivers do the same wiring in
C++ (tenzing-mcts/examples/halo_run_strategy.hpp:135-160, tenzing-dfs/examples/spmv.cu:100-120).

    import tenzing_amd as tz
    res = tz.search(g, streams=2, iters=100)                  # MCTS on the GPU, hipGraph candidates
    res = tz.search(g, streams=2, solver="dfs", sim=True)     # exhaustive, cost model, no GPU
    best = res.sims[res.best()]
    ms = tz.run(g, best.seq.json(True), streams=2)      # later: replay it, no search
"""
from __future__ import annotations

from . import _tz


def search(graph, streams: int = 2, solver: str = "mcts", iters: int = 100,
           strategy: str = "FastMin", mode: str = "graph", graph_unroll: int = 8,
           bench_iters: int = 10, target_secs: float = 0.002, race_ratio: float = 0.0,
           settle_ratio: float = 0.0,
           max_seqs: int = -1, sim: bool = False, replay: str = "", ctrl=None,
           device: int | None = None, seed: int = 0, time_budget_s: float = 0.0,
           watchdog_s: float = 0.0, symmetric_streams: bool = True, seeds=()):
    """Search the schedules of ``graph`` on ``streams`` streams and return the SearchResult.

    solver: "mcts" (``iters`` iterations, ``strategy``) or "dfs" (up to ``max_seqs``
    schedules). Candidates are timed on the GPU (``mode`` "graph": each compiled to a hipGraph
    with ``graph_unroll`` iterations per launch; "eager"), with the discrete-event model
    (``sim``) or from a results CSV (``replay``). ``ctrl``: the control plane (default: this
    process alone, or every rank when launched by torchrun); ``device``: the GPU (default: the
    local rank's). ``seeds``: schedules (Sequence or its JSON) measured before an MCTS search;
    they count as results (``seeded``), so the best is never worse than them."""
    if solver not in ("mcts", "dfs"):
        raise ValueError("solver must be 'mcts' or 'dfs'")
    if mode not in ("graph", "eager"):
        raise ValueError("mode must be 'graph' or 'eager'")
    if ctrl is None:
        from .parallel import init_ctrl

        ctrl = init_ctrl()
    plat = _tz.Platform(streams, symmetric_streams=symmetric_streams)
    bo = _tz.BenchOpts(n_iters=bench_iters, max_retries=3, target_secs=target_secs,
                       race_ratio=race_ratio, settle_ratio=settle_ratio)
    rt = None
    if replay:
        bench = _tz.CsvBenchmarker(replay, graph)
    elif sim:
        bench = _tz.SimBenchmarker(streams)
    else:
        if device is None:
            from .parallel import select_device

            device = select_device()
        if device < 0:
            raise RuntimeError("no GPU visible: pass sim=True or replay=<csv>")
        rt = _tz.HipRuntime(device=device, n_streams=streams,
                            mode=_tz.ExecMode.Graph if mode == "graph" else _tz.ExecMode.Eager,
                            watchdog_s=watchdog_s, graph_unroll=graph_unroll)
        bench = _tz.EmpiricalBenchmarker(rt, ctrl)
    if solver == "dfs":
        o = _tz.DfsOpts()
        o.max_seqs = max_seqs
        o.bench = bo
        res = _tz.dfs_explore(graph, plat, bench, ctrl, o)
    else:
        o = _tz.MctsOpts()
        o.n_iters = iters
        o.strategy = strategy
        o.seed = seed
        o.time_budget_s = time_budget_s
        o.bench = bo
        if seeds:
            idx = _tz.OpIndex(graph)
            o.seed_schedules = [s if isinstance(s, _tz.Sequence) else idx.sequence_from_json(s)
                                for s in seeds]
        res = _tz.mcts_explore(graph, plat, bench, ctrl, o)
    del bench, rt  # the runtime (and its streams) goes before the caller's tensors
    return res


def run(graph, schedule, streams: int, iters: int = 100, warmup: int = 10, mode: str = "graph",
        graph_unroll: int = 10, device: int | None = None, ctrl=None) -> float:
    """Run a found schedule of ``graph`` without searching and return milliseconds per
    iteration (max over ranks). ``schedule`` is a Sequence or its JSON (``seq.json(True)``, e.g.
    read back from a file); it is first proven race-free on the graph it executes."""
    import json as _json
    import time

    if not isinstance(schedule, _tz.Sequence):
        text = schedule if isinstance(schedule, str) else _json.dumps(schedule)
        schedule = _tz.OpIndex(graph).sequence_from_json(text)
    bad = _tz.verify(schedule, _tz.resolve_graph(graph, schedule), streams)
    if bad:
        raise ValueError("schedule is not race-free on this graph: " + "; ".join(bad[:5]))
    if ctrl is None:
        from .parallel import init_ctrl

        ctrl = init_ctrl()
    if device is None:
        from .parallel import select_device

        device = select_device()
    if device < 0:
        raise RuntimeError("no GPU visible")
    rt = _tz.HipRuntime(device=device, n_streams=streams,
                        mode=_tz.ExecMode.Graph if mode == "graph" else _tz.ExecMode.Eager,
                        graph_unroll=graph_unroll)
    rt.prepare(schedule)
    rt.precompile(warmup)
    rt.run(warmup)
    rt.precompile(iters)  # the remainder of the unroll as one graph, compiled before timing
    rt.device_sync()
    ctrl.barrier()
    t0 = time.perf_counter()
    rt.run(iters)
    rt.device_sync()
    dt = ctrl.allreduce_max([time.perf_counter() - t0])[0]
    del rt
    return dt / max(iters, 1) * 1e3


def greedy_schedule(graph, platform, prefer=None, stream_for=None, remove_redundant: bool = True):
    """One complete, race-free schedule of ``graph`` built by walking the decision tree greedily.

    ``prefer`` maps a ChoiceOp name to the name of the alternative to take; a choice named by no
    entry takes the first alternative whose name matches an entry of ``prefer["*"]`` (a list of
    substrings, e.g. ``["allfused", "fused"]``) or else its first one. ``stream_for(op_name)``
    picks the stream of each GPU op (default: stream 0). Ops execute in graph order, syncs as the
    synchronizer requires. Used to seed a search with one known schedule per alternative (for
    example one per transport), so every alternative is measured at least once.

    Returns the Sequence (its redundant synchronizations removed unless ``remove_redundant`` is
    False).
    """
    prefer = dict(prefer or {})
    patterns = list(prefer.pop("*", []))
    st = _tz.State(graph, platform)
    while not st.complete():
        ds = st.get_decisions()
        if not ds:
            raise RuntimeError("greedy_schedule: dead end (no decision, schedule incomplete)")
        g = st.graph
        pick = None
        for d in ds:
            if d.kind == "Expand":
                pick = d
                break
        if pick is None:
            for d in ds:
                if d.kind != "Choose":
                    continue
                op = g.op(d.node)
                names = [c.name for c in op.choices()]
                want = prefer.get(op.name)
                if want is None:
                    for p in patterns:
                        hit = [k for k, n in enumerate(names) if p in n]
                        if hit:
                            want = names[hit[0]]
                            break
                k = names.index(want) if want in names else 0
                if d.choice == k:
                    pick = d
                    break
        if pick is None:
            for d in ds:
                if d.kind == "Assign":
                    s = stream_for(g.op(d.node).name) if stream_for else 0
                    if d.stream == s:
                        pick = d
                        break
            if pick is None:
                # stream not offered yet (symmetric streams offer used ones plus one fresh one):
                # take the highest offered stream not above the wish
                assigns = [d for d in ds if d.kind == "Assign"]
                if assigns:
                    node = assigns[0].node
                    want = stream_for(g.op(node).name) if stream_for else 0
                    cands = [d for d in assigns if d.node == node]
                    below = [d for d in cands if d.stream <= want]
                    pick = max(below, key=lambda d: d.stream) if below else cands[0]
        if pick is None:
            ex = [d for d in ds if d.kind == "Execute"]
            graph_ops = [d for d in ex if d.node >= 0]
            pick = (graph_ops or ex)[0]
        st = st.apply(pick)
    seq = st.sequence
    if remove_redundant:
        seq, _ = _tz.remove_redundant_syncs(seq, st.graph, platform.n_streams)
    return seq


def choice_alternatives(graph, name: str):
    """Names of the alternatives of the ChoiceOp ``name`` anywhere in ``graph`` (compound
    sub-graphs and nested choices included), [] if there is none."""
    seen = set()

    def walk(g):
        for v in g.vertices():
            op = g.op(v)
            if op.name == name and hasattr(op, "choices"):
                return [c.name for c in op.choices()]
            if op.name in seen:
                continue
            seen.add(op.name)
            subs = []
            if hasattr(op, "graph"):
                subs.append(op.graph())
            if hasattr(op, "choices"):
                for c in op.choices():
                    if hasattr(c, "graph"):
                        subs.append(c.graph())
            for sg in subs:
                r = walk(sg)
                if r:
                    return r
        return []

    return walk(graph)
