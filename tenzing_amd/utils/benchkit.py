"""Pieces of ``bench.py`` that are worth testing on their own.

* ``branch_probe`` / ``choose_pad``: does HIP's graph executor run three independent branches of
  a captured schedule at once on this box, with this runtime's stream padding? (round 4 found a
  3-branch graph serializing unless the process owns spare streams: 449 vs 232 us,
  ``profiles/archive/r4_capture/README.md:42-57``). The bench probes the runtime it is about to search
  with, retries other paddings if the branches serialize, and records what it found.
* ``timed_replay``: the timing contract of every number the bench reports (W untimed warm-up
  iterations, then K timed ones bracketed by barrier + device sync, max over ranks).
* ``search_record``: a short search of another workload, its winner verified and timed the same
  way as the headline -- the bench's sub-records (the reference's XYZQ halo layout, BASELINE
  configs 2 and 5) so that the driver's own run observes them.

Reference: the drivers time with MPI_Wtime around MPI_Barrier'd batches, max over ranks
(src/benchmarker.cpp:83-119); tenzing-mcts/examples/spmv_run_strategy.cuh:44-68 and
halo_run_strategy.hpp:42-49 give the sub-record configurations.
"""
from __future__ import annotations

import json
import sys
import time

# which transport an op of a halo schedule belongs to (by op-name prefix)
VIA_PREFIXES = (("direct", "he_direct_"), ("rccl", "he_shift_"), ("ipc", "he_put_"),
                ("ipc_wide", "he_putw_"),
                ("sdma", "he_copyput_"), ("memcpy", "he_mcput_"), ("relay", "he_rl"),
                ("hostsplit", "he_hs"), ("host", "he_hostxfer"))


def schedule_via(names):
    """Transports a schedule uses, in VIA_PREFIXES order."""
    return [t for t, key in VIA_PREFIXES if any(n.startswith(key) for n in names)]


def remote_via(names):
    """The transport of the remote directions ("mixed": kernel and copy-engine puts at once;
    relay and host split carry their share in percent, e.g. "relay20", "hostsplit35")."""
    via = [t for t in schedule_via(names) if t != "direct"]
    if "ipc" in via and "sdma" in via:
        return "mixed"
    if not via:
        return None
    if via[0] in ("relay", "hostsplit"):
        key = "he_rl" if via[0] == "relay" else "he_hs"
        share = next(n[len(key):].split("_")[0] for n in names if n.startswith(key))
        return via[0] + share
    return via[0]


BRANCH_PREFIX = "branch_probe"


def _busy_graph(tz, branches: int, us: float):
    g = tz.Graph()
    for i in range(branches):
        op = tz.BusyKernelOp(f"{BRANCH_PREFIX}{i}", us)
        g.start_then(op)
        g.then_finish(op)
    return g


def branch_probe(tz, rt, branches: int = 3, us: float = 200.0, iters: int = 10, unroll: int = 10):
    """Microseconds per run of ``branches`` independent ``us``-long single-workgroup kernels, one
    per stream of ``rt`` (compiled the way the runtime compiles every schedule), and of one such
    kernel alone. ``ratio`` = all / one: about 1 when the branches run at once, about
    ``branches`` when they serialize.

    Two forms: one schedule copy per hipGraphLaunch (``ratio``), and ``unroll`` copies captured
    into one graph (``unrolled``), which is how the search and the timing replay a schedule.
    Device timestamps (``scripts/stagger_probe.hip``, profiles/r5_branch/) show why both are
    kept: with one copy per launch, HIP starts each further branch 4-10 us after the previous one
    and the next launch 18-27 us after the join; inside an unrolled graph the branches start
    within ~1 us of each other and a join costs 5-8 us. So the kernels are long (200 us) for the
    one-copy ratio to tell overlap from serialization. The runtime's mode and unroll are
    restored; None if the runtime cannot build the graph."""
    from ..search import greedy_schedule

    if rt.num_streams() < branches:
        return None
    mode, old_unroll = rt.mode, rt.graph_unroll
    rt.set_mode(tz.ExecMode.Graph)

    def per_run(k, u):
        rt.set_graph_unroll(u)
        g = _busy_graph(tz, k, us)
        seq = greedy_schedule(g, tz.Platform(rt.num_streams(), symmetric_streams=False),
                              stream_for=lambda n: int(n[len(BRANCH_PREFIX):]))
        rt.prepare(seq)
        if rt.effective_mode != tz.ExecMode.Graph:
            return None
        n = iters * u
        rt.run(u)
        rt.device_sync()
        t0 = time.perf_counter()
        rt.run(n)
        rt.device_sync()
        return (time.perf_counter() - t0) / n * 1e6

    try:
        one = per_run(1, 1)
        many = per_run(branches, 1)
        one_u = per_run(1, unroll) if unroll > 1 else None
        many_u = per_run(branches, unroll) if unroll > 1 else None
    finally:
        rt.set_mode(mode)
        rt.set_graph_unroll(old_unroll)
    if not one or not many:
        return None
    out = {"branches": branches, "kernel_us": us, "one_us": round(one, 1),
           "all_us": round(many, 1), "ratio": round(many / one, 3),
           "extra_us_per_branch": round((many - one) / max(1, branches - 1), 1)}
    if one_u and many_u:
        out["unrolled"] = {"unroll": unroll, "one_us": round(one_u, 1), "all_us": round(many_u, 1),
                           "ratio": round(many_u / one_u, 3)}
    return out


def choose_pad(make_rt, probe, pads, threshold: float = 1.5, margin: float = 0.9):
    """Runtime whose graph branches run concurrently: ``make_rt(pad)`` builds a runtime with that
    stream padding (None: the default), ``probe(rt)`` returns its branch probe (a dict with
    ``ratio``, or None). The first padding whose ratio is at most ``threshold`` is kept;
    otherwise the one with the lowest ratio if that is below ``margin`` times the first
    padding's (a clear gain, not probe noise), else the first (built again if it is not the last
    one probed).

    The ratio judged is the probe's ``unrolled`` one when it has it (the form the search and the
    timing replay: several schedule copies per graph launch), else its one-copy ``ratio``.

    Returns (runtime, record); the record lists every probe in order and the padding chosen."""
    def judged(r):
        if not r:
            return None
        return (r.get("unrolled") or {}).get("ratio") or r.get("ratio")

    tried = []
    best = None  # (ratio, pad)
    rt = None
    for pad in pads:
        rt = None  # the previous runtime (and its streams) goes before the next is made
        rt = make_rt(pad)
        r = probe(rt)
        used = rt.pad_streams if hasattr(rt, "pad_streams") else pad
        tried.append({"pad_streams": used, "probe": r})
        ratio = judged(r)
        if ratio is not None and ratio <= threshold:
            return rt, {"pad_streams": used, "serialized": False, "tried": tried,
                        "threshold": threshold}
        if ratio is not None and (best is None or ratio < best[0]):
            best = (ratio, pad, used)
    if best is None:  # the probe could not run at all: keep the last runtime, say so
        return rt, {"pad_streams": tried[-1]["pad_streams"] if tried else None,
                    "serialized": None, "tried": tried, "threshold": threshold}
    first = judged(tried[0]["probe"])
    if first is not None and best[0] > margin * first:  # no padding is clearly better
        best = (first, pads[0], tried[0]["pad_streams"])
    if best[1] != pads[-1]:
        rt = None
        rt = make_rt(best[1])
    return rt, {"pad_streams": best[2], "serialized": True, "tried": tried,
                "threshold": threshold}


def timed_replay(tz, rt, ctrl, seq, mode, steps: int, warmup: int):
    """(seconds for ``steps`` iterations of ``seq`` in ``mode``, max over ranks, or None if the
    mode could not be prepared on some rank; the mode that ran). ``warmup`` untimed iterations
    first; the timed ones are bracketed by device sync + barrier on both sides."""
    rt.set_mode(mode)
    ok = 1.0
    try:
        rt.prepare(seq)
        ok = 1.0 if rt.effective_mode == mode else 0.0
    except Exception:  # noqa: BLE001 (agreed below: every rank falls back together)
        ok = 0.0
    if ctrl.allreduce_max([1.0 - ok])[0] > 0:
        rt.set_mode(tz.ExecMode.Eager)
        rt.prepare(seq)
        return None, tz.ExecMode.Eager
    # a step count that is no multiple of the graph unroll: its remainder runs as one graph too
    # (compiled here, outside the timed region), not as one-iteration launches
    def precompile(n):
        try:
            rt.precompile(n)
        except Exception as e:  # noqa: BLE001 (then the remainder runs as one-iteration launches)
            print(f"timed_replay: no remainder graph for {n} steps: {e}", file=sys.stderr)

    if hasattr(rt, "precompile"):
        precompile(warmup)
    rt.run(warmup)
    if hasattr(rt, "precompile"):
        precompile(steps)
    rt.device_sync()
    ctrl.barrier()
    t0 = time.perf_counter()
    rt.run(steps)
    rt.device_sync()
    ctrl.barrier()
    dt = time.perf_counter() - t0
    return ctrl.allreduce_max([dt])[0], rt.effective_mode


def search_record(tz, ctrl, rt, graph, streams: int, verify, steps: int, warmup: int,
                  mcts_iters: int = 40, bench_iters: int = 6, target_secs: float = 0.002,
                  search_unroll: int = 10, graph_unroll: int = 20, seed: int = 0,
                  time_budget_s: float = 30.0, strategy: str = "FastMin", rerank: int = 4,
                  seeds=(), bench=None):
    """Search ``graph`` briefly (MCTS, hipGraph candidates, racing and settling as the headline),
    re-rank the ``rerank`` best distinct candidates interleaved, verify the winner with
    ``verify(seq) -> bad count`` (the next finalist if it fails), then time it eagerly and as a
    hipGraph exactly as the headline is timed. ``seeds``: schedules measured before the search
    (they count as results); ``bench``: the benchmarker (default: an EmpiricalBenchmarker on
    ``rt``; tests pass a simulator). Every rank must call it together. Returns the sub-record
    dict."""
    t_start = time.time()
    plat = tz.Platform(streams)
    rt.set_mode(tz.ExecMode.Graph)
    rt.set_graph_unroll(search_unroll)
    if bench is None:
        bench = tz.EmpiricalBenchmarker(rt, ctrl)
    o = tz.MctsOpts()
    o.n_iters = mcts_iters
    o.time_budget_s = time_budget_s
    o.strategy = strategy
    o.seed = seed
    o.bench = tz.BenchOpts(n_iters=bench_iters, max_retries=3, target_secs=target_secs,
                           race_ratio=1.25, settle_ratio=0.03)
    if seeds and ctrl.rank == 0:
        o.seed_schedules = list(seeds)
    res = tz.mcts_explore(graph, plat, bench, ctrl, o)
    # only rank 0 holds the results: its finalists go to every rank (by op name), so that all
    # ranks re-rank, verify and time the same schedules in the same collectives
    payload = ""
    if ctrl.rank == 0:
        order = sorted(range(len(res.sims)), key=lambda i: res.sims[i].res.pct10)
        top, keys = [], set()
        for i in order:
            k = res.sims[i].seq.canonical_key()
            if k not in keys:
                keys.add(k)
                top.append(i)
            if len(top) >= max(1, rerank):
                break
        payload = json.dumps({"seqs": [res.sims[i].seq.json() for i in top],
                              "pct10": [res.sims[i].res.pct10 for i in top],
                              "n": len(res.sims), "failed": res.failed})
    payload = json.loads(ctrl.bcast(payload, 0).decode())
    rec = {"mcts_candidates": payload["n"], "mcts_skipped": payload["failed"],
           "search_wall_s": round(res.wall_s, 3), "seeded": len(seeds)}
    if not payload["seqs"]:
        rec["error"] = "the search measured no candidate"
        return rec
    index = tz.OpIndex(graph)
    cands = [index.sequence_from_json(j) for j in payload["seqs"]]
    rec["search_best_pct10_ms"] = payload["pct10"][0] * 1e3
    ranked = list(range(len(cands)))
    if len(cands) > 1:
        ro = tz.BenchOpts(n_iters=bench_iters, max_retries=1, target_secs=target_secs)
        if hasattr(bench, "benchmark_many"):  # interleaved
            rr = bench.benchmark_many(cands, ro, seed)
        else:
            rr = [bench.benchmark(c, ro) for c in cands]
        ranked = sorted(range(len(rr)), key=lambda i: rr[i].pct10)
        rec["rerank_pct10_ms"] = [round(r.pct10 * 1e3, 5) for r in rr]
    rt.set_mode(tz.ExecMode.Eager)
    best, bad, rejected = None, None, 0
    for k in ranked:
        b = verify(cands[k])
        if b == 0:
            best, bad = cands[k], 0
            break
        rejected += 1
    if best is None:
        best, bad = cands[ranked[0]], int(verify(cands[ranked[0]]))
    rec["verified_bad"] = int(bad)
    rec["verify_rejected"] = rejected
    t_e, _ = timed_replay(tz, rt, ctrl, best, tz.ExecMode.Eager, steps, warmup)
    rt.set_graph_unroll(graph_unroll)
    t_g, eff = timed_replay(tz, rt, ctrl, best, tz.ExecMode.Graph, steps, warmup)
    graph_ok = t_g is not None and eff == tz.ExecMode.Graph
    use_graph = graph_ok and t_g < t_e
    t = t_g if use_graph else t_e
    rec.update({"ms_per_step": t / steps * 1e3, "timed_mode": "hipgraph" if use_graph else "eager",
                "eager_ms_per_step": t_e / steps * 1e3,
                "graph_ms_per_step": (t_g / steps * 1e3) if graph_ok else None,
                "schedule_ops": len(best), "steps": steps, "warmup": warmup,
                "schedule_gpu_ops": [o.name for o in best.ops() if o.op_class == "BoundGpu"],
                "wall_s": round(time.time() - t_start, 2)})
    # correctness after the timed iterations too (the sub-record's workload decides what a
    # bad result is)
    after = verify(None)
    rec["verified_bad_after_timing"] = int(after)
    return rec


def _main(argv=None) -> int:
    """``python -m tenzing_amd.utils.benchkit probe [--streams 4] [--pad -1] [--us 50]``: one JSON
    line per branch count (2, 3, 4) with the graph-branch probe of a fresh runtime (for A/B of
    the HIP runtime's environment knobs, one process per setting)."""
    import argparse
    import json
    import os

    ap = argparse.ArgumentParser(prog="python -m tenzing_amd.utils.benchkit")
    ap.add_argument("cmd", choices=["probe"])
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--pad", type=int, default=-1)
    ap.add_argument("--us", type=float, default=200.0)
    a = ap.parse_args(argv)
    import tenzing_amd as tz

    rt = tz.HipRuntime(device=0, n_streams=a.streams, pad_streams=a.pad)
    env = {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_HIP", "GPU_MAX_HW", "HIP_", "TZ_PAD"))}
    for k in (2, 3, 4):
        if k > a.streams:
            continue
        print(json.dumps({"env": env, "pad_streams": rt.pad_streams,
                          "probe": branch_probe(tz, rt, branches=k, us=a.us)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
