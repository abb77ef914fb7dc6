"""``python -m tenzing_amd`` — search / run / replay / rules / env.

  python -m tenzing_amd search --workload halo --solver mcts --strategy FastMin --iters 100
  python -m tenzing_amd search --workload spmv --solver dfs --max-seqs 15000 --csv spmv.csv
  python -m tenzing_amd search --workload halo --replay halo.csv      # MCTS on recorded timings
  python -m tenzing_amd search --workload fused --sim                  # hardware-free (cost model)
  python -m tenzing_amd search --workload halo --save-best best.json   # search once ...
  python -m tenzing_amd run best.json --iters 1000                     # ... deploy many times
  python -m tenzing_amd rules spmv.csv --out spmv_                     # design rules
  python -m tenzing_amd env --topology

Multi-GPU: ``torchrun --nproc-per-node 8 -m tenzing_amd search ...`` (one process per GPU).
Reference drivers: tenzing-mcts/examples/{halo,spmv}_*.cu, tenzing-dfs/examples/spmv.cu,
tenzing-mcts/examples/mcts_csv_*.cu (CSV replay, not built in the reference).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _build_workload(a, ctrl, device, setup):
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused, build_halo, build_spmv

    grid = ()
    if a.rank_grid:
        try:
            grid = tuple(int(v) for v in a.rank_grid.lower().split("x"))
        except ValueError:
            grid = ()
        if len(grid) != 3:
            raise SystemExit("--rank-grid must look like 2x2x2")
    hc = HaloConfig(n=a.halo_n, nq=a.nq, ghost=a.ghost, neighbors=a.neighbors, order=a.order,
                    fuse=a.fuse, transport=a.transport, stencil=a.stencil, relay=a.relay,
                    relay_fracs=tuple(float(f) for f in a.relay_fracs.split(",")),
                    hostsplit=a.hostsplit,
                    hostsplit_fracs=tuple(float(f) for f in a.hostsplit_fracs.split(",")),
                    hostsplit_chunks=a.hostsplit_chunks, rank_grid=grid,
                    wide_puts=a.wide_puts, wide_put_blocks=a.wide_put_blocks,
                    ipc_grid=None if a.ipc_grid == "auto" else int(a.ipc_grid),
                    copy_puts=a.copy_puts == "on", copy_engines=a.copy_engines,
                    move_pairs=a.move_pairs == "on",
                    grid_memory={"auto": -1, "coarse": 0, "fine": 1}[a.grid_memory])
    sc = SpmvConfig(m=a.spmv_m, form=a.spmv_form, transport=a.spmv_transport,
                    matrix=a.spmv_matrix, library=a.spmv_library, distribute=a.spmv_distribute)
    if a.workload == "halo":
        h, g = build_halo(hc, ctrl, device, setup)
        return g, {"halo": h}
    if a.workload == "spmv":
        s, g = build_spmv(sc, ctrl, device, setup)
        return g, {"spmv": s}
    if a.workload == "fused":
        h, s, g = build_fused(hc, sc, ctrl, device, setup, horizontal=a.horizontal == "on")
        return g, {"halo": h, "spmv": s}
    if a.workload == "noop":
        # reference test/test_noop_graph.cpp: Start -> op1 -> Finish (here: `--noop-width`
        # independent no-ops, so DFS has orderings and stream choices to enumerate)
        g = tz.Graph()
        for i in range(a.noop_width):
            op = tz.NoOp(f"op{i + 1}")
            g.start_then(op)
            g.then_finish(op)
        return g, {}
    if a.workload == "diamond":
        g = tz.Graph()
        k = [tz.BusyKernelOp(f"k{i}", us) for i, us in enumerate((20, 100, 100, 20), 1)]
        g.start_then(k[0])
        g.then(k[0], k[1])
        g.then(k[0], k[2])
        g.then(k[1], k[3])
        g.then(k[2], k[3])
        g.then_finish(k[3])
        return g, {}
    raise SystemExit(f"unknown workload {a.workload}")


def _link_record(path: str) -> dict:
    """the last bench record holding a ``link_probe`` in a file (JSON lines, one document, or
    any JSON nesting records)"""
    from tenzing_amd.parallel.linkmodel import load_records

    recs = load_records(path)
    if not recs:
        raise SystemExit(f"--link-model: no record with a link_probe in {path}")
    return recs[-1]


def cmd_search(a) -> int:
    import tenzing_amd as tz
    from tenzing_amd.parallel import init_ctrl, select_device

    ctrl = init_ctrl()
    if ctrl.rank == 0:
        # version + command line, like the reference's reproduce::dump_with_cli (stderr keeps
        # stdout for results)
        print(tz._tz.reproduce_json(sys.argv), file=sys.stderr, flush=True)
    if a.workload == "noop":
        a.host = True  # no GPU op in the graph: time it on the host executor
    hw = not (a.sim or a.replay or a.host)
    device = select_device() if hw else -1
    if hw and device < 0:
        raise SystemExit("no GPU visible: use --sim or --replay")
    if hw and a.bind_cpus:
        from tenzing_amd.utils.env import bind_local_cpus

        bind_local_cpus(device)
    g, wl = _build_workload(a, ctrl, device, hw)
    if a.dump_graph and ctrl.rank == 0:
        with open(a.dump_graph, "w") as f:
            f.write(g.dump_graphviz(a.workload))
    distinct = a.cu_partition or bool(a.stream_priorities)
    # CU-masked or prioritized streams are distinguishable resources: binding an op to stream 0
    # or 1 is then a real choice, so the symmetric-stream pruning is off
    plat = tz.Platform(a.streams, symmetric_streams=not distinct)
    bo = tz.BenchOpts(n_iters=a.bench_iters, max_retries=a.max_retries, target_secs=a.target_secs,
                      device_timer=a.device_timer, race_ratio=a.race_ratio,
                      settle_ratio=a.settle_ratio)
    rt = None
    if a.replay:
        bench = tz.CsvBenchmarker(a.replay, g)
    elif a.host:
        rt = tz.HostExecutor(a.streams)
        bench = tz.EmpiricalBenchmarker(rt, ctrl)
    elif a.sim:
        if a.link_model is not None:
            # per-peer link / engine rates (a multi-GPU bench record's, or the defaults)
            from tenzing_amd.parallel.linkmodel import link_sim_params
            rec = _link_record(a.link_model) if a.link_model else {}
            p = link_sim_params(rec.get("link_probe"), rec.get("link_matrix"),
                                graph=a.mode == "graph")
        else:
            p = tz.SimParams()
            p.graph = a.mode == "graph"  # time candidates as a replayed hipGraph (measured costs)
        # every rank simulates its own graph; the time of a schedule is the max over ranks
        bench = tz.SimBenchmarker(a.streams, p, ctrl)
    else:
        mode = tz.ExecMode.Graph if a.mode == "graph" else tz.ExecMode.Eager
        prio = [int(x) for x in a.stream_priorities.split(",")] if a.stream_priorities else []
        rt = tz.HipRuntime(device=device, n_streams=a.streams, priorities=prio,
                           cu_partition=a.cu_partition, mode=mode, watchdog_s=a.watchdog,
                           graph_unroll=a.graph_unroll)
        bench = tz.EmpiricalBenchmarker(rt, ctrl)
    t0 = time.time()
    if a.solver == "dfs":
        o = tz.DfsOpts()
        o.max_seqs = a.max_seqs
        o.bench = bo
        o.trap_signals = True  # SIGINT/SIGTERM: print the partial results CSV, exit 1
        res = tz.dfs_explore(g, plat, bench, ctrl, o)
    else:
        o = tz.MctsOpts()
        o.n_iters = a.iters
        o.time_budget_s = a.time_budget
        o.max_tree_nodes = a.max_tree_nodes
        o.strategy = a.strategy
        o.seed = a.seed
        o.expand_rollout = not a.no_expand_rollout
        o.dump_tree = a.dump_tree
        o.bench = bo
        o.trap_signals = True
        if a.seed_schedule and ctrl.rank == 0:
            # a `--save-best` document, or a bare schedule (JSON array of ops)
            seeds = []
            for path in a.seed_schedule:
                with open(path) as f:
                    doc = json.load(f)
                sched = doc["schedule"] if isinstance(doc, dict) else doc
                seeds.append(tz.OpIndex(g).sequence_from_json(json.dumps(sched)))
            o.seed_schedules = seeds
        if a.checkpoint:
            o.checkpoint_path = a.checkpoint
            o.checkpoint_every = 10
        if a.resume:
            o.resume_path = a.resume
        res = tz.mcts_explore(g, plat, bench, ctrl, o)
    if ctrl.rank == 0:
        if a.csv:
            with open(a.csv, "w") as f:
                f.write(res.dump_csv())
        if a.jsonl:
            with open(a.jsonl, "w") as f:
                f.write(res.dump_jsonl())
        b = res.best()
        summary = {"workload": a.workload, "solver": a.solver, "ranks": ctrl.size,
                   "streams": a.streams, "candidates": len(res.sims), "search_wall_s": res.wall_s,
                   "stop_reason": res.stop_reason, "counters": res.counters(),
                   "skipped": res.failed, "dead_domains": list(res.dead_domains),
                   "pruned_dead": res.pruned_dead, "elapsed_s": time.time() - t0}
        if a.sim:
            summary["sim"] = {"graph_replay": a.mode == "graph", "link_model": a.link_model is not None,
                              "link_record": a.link_model or None}
        if b >= 0:
            summary["best_pct10_ms"] = res.sims[b].res.pct10 * 1e3
            summary["best_schedule"] = json.loads(res.sims[b].seq.json())
            if a.save_best:
                _save_best(a, tz, ctrl, res.sims[b])
        print(json.dumps(summary))
    if a.trace_best:
        _trace_best(a, tz, ctrl, g, res, rt)
    return 0


# search options that describe the workload and the platform (what `run` needs to rebuild the
# graph a saved schedule refers to); solver and measurement options are not part of it
# (the same keys, with the same meaning, as `tz-search --save-best` writes)
_WORKLOAD_KEYS = ("workload", "noop_width", "streams", "halo_n", "nq", "ghost", "neighbors",
                  "order", "fuse", "transport", "relay", "relay_fracs", "hostsplit",
                  "hostsplit_fracs", "hostsplit_chunks", "wide_puts", "wide_put_blocks",
                  "ipc_grid", "copy_puts", "copy_engines", "move_pairs", "horizontal",
                  "stencil", "rank_grid",
                  "spmv_m", "spmv_matrix", "spmv_form", "spmv_transport", "spmv_library",
                  "spmv_distribute",
                  "cu_partition", "stream_priorities")


def _saved_args(args: dict):
    """The search options of a saved document, parsed like a command line (so values written
    as strings by the native CLI get the same types)."""
    argv = ["search"]
    for k, v in args.items():
        if k not in _WORKLOAD_KEYS:
            continue
        if k == "workload" and v == "halo+spmv":  # the native CLI's name for it
            v = "fused"
        flag = "--" + k.replace("_", "-")
        if isinstance(v, bool):
            if v:
                argv.append(flag)
        else:
            argv.append(f"{flag}={v}")
    return _parser().parse_args(argv)


def _save_best(a, tz, ctrl, sim) -> None:
    """The best schedule plus everything needed to run it again: the workload options, the
    rank count and the reference's schedule JSON (ops by name, `in_graph` flags)."""
    doc = {"tenzing_amd": tz.__version__, "ranks": ctrl.size, "mode": a.mode,
           "pct10_ms": sim.res.pct10 * 1e3,
           "args": {k: getattr(a, k) for k in _WORKLOAD_KEYS},
           "schedule": json.loads(sim.seq.json(True))}
    with open(a.save_best, "w") as f:
        json.dump(doc, f, indent=1)


def load_schedule(doc: dict, ctrl, device: int, setup: bool):
    """(workload options, graph, workload objects, sequence) of a `--save-best` document. The
    workload is rebuilt from the saved options, the schedule is rebuilt by op name and checked
    race-free against the graph it executes (choices resolved, compounds expanded)."""
    import tenzing_amd as tz

    w = _saved_args(doc["args"])
    # a schedule that uses the wide put needs it offered again, wherever it runs now ("auto"
    # decides by the devices of this launch)
    if hasattr(w, "wide_puts") and "he_putw_" in json.dumps(doc["schedule"]):
        w.wide_puts = "on"
    g, wl = _build_workload(w, ctrl, device, setup)
    if setup and "halo" in wl and "he_putw_" in json.dumps(doc["schedule"]) \
            and not wl["halo"].uses_wide_puts():
        raise SystemExit("the saved schedule uses wide IPC puts (he_putw_*), which this launch "
                         "does not offer: " + wl["halo"].transport_report()["wide_put"] +
                         " (e.g. the put block cap equal to --wide-put-blocks, or its preflight "
                         "failed on this node)")
    seq = tz.OpIndex(g).sequence_from_json(json.dumps(doc["schedule"]))
    bad = tz.verify(seq, tz.resolve_graph(g, seq), w.streams)
    if bad:
        raise SystemExit("schedule is not race-free on this graph: " + "; ".join(bad[:5]))
    return w, g, wl, seq


def cmd_run(a) -> int:
    """Run a saved schedule without searching: rebuild the workload, rebuild the sequence by op
    name, prove it race-free on the graph it executes, check the results once, then time it."""
    import tenzing_amd as tz
    from tenzing_amd.parallel import init_ctrl, select_device

    with open(a.schedule) as f:
        doc = json.load(f)
    ctrl = init_ctrl()
    if ctrl.size != doc["ranks"]:
        raise SystemExit(f"schedule was searched on {doc['ranks']} ranks, this run has {ctrl.size}")
    if doc["args"].get("workload") == "noop":
        raise SystemExit("run: the no-op workload has no GPU work")
    device = select_device()
    if device < 0:
        raise SystemExit("run: no GPU visible")
    w, g, wl, seq = load_schedule(doc, ctrl, device, True)
    mode = a.mode or doc.get("mode", "graph")
    prio = [int(x) for x in w.stream_priorities.split(",")] if w.stream_priorities else []
    rt = tz.HipRuntime(device=device, n_streams=w.streams, priorities=prio,
                       cu_partition=w.cu_partition,
                       mode=tz.ExecMode.Graph if mode == "graph" else tz.ExecMode.Eager,
                       watchdog_s=a.watchdog, graph_unroll=a.graph_unroll)
    if "halo" in wl:
        wl["halo"].init_grid()
    if "spmv" in wl:
        wl["spmv"].reset_y()
    rt.device_sync()
    rt.prepare(seq)
    rt.run(1)
    rt.device_sync()
    out = {"schedule": a.schedule, "workload": w.workload, "ranks": ctrl.size,
           "streams": w.streams, "mode": "graph" if rt.effective_mode == tz.ExecMode.Graph
           else "eager"}
    ok = True
    if "halo" in wl:
        out["halo_bad_cells"] = int(ctrl.allreduce_sum([float(wl["halo"].check_grid())])[0])
        ok &= out["halo_bad_cells"] == 0
        if a.torch_model == "on":
            # once more against the independent torch model (tenzing_amd/utils/halo_ref.py)
            from tenzing_amd.utils.halo_ref import check_prepared

            out["torch_model_check"] = check_prepared(wl["halo"], rt, ctrl, device)
            ok &= out["torch_model_check"]["bad_cells"] == 0
    if "spmv" in wl:
        out["spmv_max_rel_err"] = ctrl.allreduce_max([wl["spmv"].check()])[0]
        ok &= out["spmv_max_rel_err"] < 1e-4
    rt.precompile(a.warmup)
    rt.run(a.warmup)
    rt.precompile(a.iters)  # the remainder of the unroll as one graph, compiled before timing
    rt.device_sync()
    ctrl.barrier()
    t0 = time.perf_counter()
    rt.run(a.iters)
    rt.device_sync()
    dt = ctrl.allreduce_max([time.perf_counter() - t0])[0]
    out["iters"] = a.iters
    out["ms_per_iter"] = dt / max(a.iters, 1) * 1e3
    out["searched_pct10_ms"] = doc.get("pct10_ms")
    out["correct"] = bool(ok)
    if ctrl.rank == 0:
        print(json.dumps(out))
    return 0 if ok else 1


def _trace_best(a, tz, ctrl, g, res, rt) -> None:
    """Timeline of the best schedule as Chrome trace-event JSON (chrome://tracing, Perfetto):
    measured per-op device times on hardware (every rank runs it, each writes its own file),
    the discrete-event model's timeline with --sim."""
    msg = ""
    if ctrl.rank == 0 and res.best() >= 0:
        msg = res.sims[res.best()].seq.json(True)
    msg = ctrl.bcast(msg, 0).decode()
    if not msg:
        return
    seq = tz.OpIndex(g).sequence_from_json(msg)
    if a.sim:
        ex = tz.SimExecutor(a.streams)
        ex.run_once(seq)
        spans = [(n, st, 0, t0, t1) for n, st, t0, t1 in ex.trace()]
    elif isinstance(rt, tz.HipRuntime):
        spans = rt.trace(seq, a.trace_iters)
    else:
        if ctrl.rank == 0:
            print("--trace-best needs a GPU run or --sim", file=sys.stderr)
        return
    path = a.trace_best
    if ctrl.size > 1:
        root, ext = os.path.splitext(path)
        path = f"{root}.r{ctrl.rank}{ext or '.json'}"
    with open(path, "w") as f:
        f.write(tz._tz.chrome_trace(spans))


def cmd_rules(a) -> int:
    from tenzing_amd.utils import postprocess

    return postprocess.main([a.results] + (["--out", a.out] if a.out else []) +
                            (["--plots"] if a.plots else []))


def cmd_env(a) -> int:
    from tenzing_amd.utils.env import env_report

    import tenzing_amd as tz

    print(json.dumps(env_report(0 if tz.hip_device_count() else None, a.topology), indent=1))
    return 0


def cmd_links(a) -> int:
    """The fabric between the ranks of this launch (one process per GPU, started like bench.py):
    the all-pairs link matrix and each peer's device facts, as one JSON line from rank 0."""
    import tenzing_amd as tz
    from tenzing_amd.parallel import init
    from tenzing_amd.parallel.topology import peer_device_facts

    ctrl, dev = init()
    lm = tz._tz.link_matrix(ctrl, int(a.mib) << 20, a.iters)
    facts = peer_device_facts(ctrl, dev, range(ctrl.size))
    if ctrl.rank == 0:
        print(json.dumps({"ranks": ctrl.size, "link_matrix": lm, "peer_devices": facts}), flush=True)
    return 0 if ctrl.size == 1 or not lm["why"] else 1


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    return a.fn(a)


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m tenzing_amd", description=__doc__.splitlines()[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("search")
    s.add_argument("--workload", default="halo",
                   choices=["halo", "spmv", "fused", "diamond", "noop"])
    s.add_argument("--noop-width", type=int, default=1)
    s.add_argument("--host", action="store_true",
                   help="time schedules on the host executor (CPU-only graphs)")
    s.add_argument("--solver", default="mcts", choices=["mcts", "dfs"])
    s.add_argument("--strategy", default="FastMin")
    s.add_argument("--iters", type=int, default=300)
    s.add_argument("--time-budget", type=float, default=0.0)
    s.add_argument("--seed-schedule", action="append", default=[],
                   help="MCTS: measure this schedule (a --save-best document or a JSON array of "
                        "ops of this workload) before searching; repeatable")
    s.add_argument("--max-tree-nodes", type=int, default=0,
                   help="MCTS: stop once the tree holds this many nodes (0 = unlimited)")
    s.add_argument("--max-seqs", type=int, default=15000)
    s.add_argument("--streams", type=int, default=2)
    s.add_argument("--bench-iters", type=int, default=50)
    s.add_argument("--max-retries", type=int, default=10)
    s.add_argument("--target-secs", type=float, default=0.01)
    s.add_argument("--race-ratio", type=float, default=0.0,
                   help="stop measuring candidates clearly slower than this times the best so far")
    s.add_argument("--settle-ratio", type=float, default=0.0,
                   help="stop measuring a candidate once settle-min measurements agree within this ratio")
    s.add_argument("--device-timer", action="store_true",
                   help="time measurements with device events (GPU time) instead of host wall clock")
    s.add_argument("--mode", default="eager", choices=["eager", "graph"],
                   help="with --sim: graph = the hipGraph replay cost model (SimParams.graph)")
    s.add_argument("--graph-unroll", type=int, default=1,
                   help="graph mode: iterations per hipGraph launch while benchmarking")
    s.add_argument("--cu-partition", action="store_true",
                   help="give each stream a disjoint, XCD-balanced CU mask")
    s.add_argument("--stream-priorities", default="",
                   help="comma-separated HIP stream priorities, one per stream (e.g. -1,0)")
    s.add_argument("--sim", action="store_true", help="discrete-event cost model, no GPU")
    s.add_argument("--link-model", nargs="?", const="", default=None, metavar="RECORD",
                   help="with --sim: the link-aware model (per-peer xGMI / PCIe / HBM bytes over "
                        "shared link capacities); RECORD: a multi-GPU bench record whose link_probe "
                        "and link_matrix give the rates (default: built-in rates)")
    s.add_argument("--replay", default="", help="results CSV to replay instead of running")
    s.add_argument("--seed", type=int, default=0)
    s.add_argument("--no-expand-rollout", action="store_true")
    s.add_argument("--dump-tree", action="store_true")
    s.add_argument("--dump-graph", default="")
    s.add_argument("--checkpoint", default="")
    s.add_argument("--resume", default="")
    s.add_argument("--csv", default="")
    s.add_argument("--jsonl", default="")
    s.add_argument("--save-best", default="",
                   help="write the best schedule and its workload options as JSON (for `run`)")
    s.add_argument("--trace-best", default="",
                   help="write the best schedule's timeline as Chrome trace JSON (per rank)")
    s.add_argument("--trace-iters", type=int, default=2,
                   help="iterations in the --trace-best timeline")
    s.add_argument("--watchdog", type=float, default=30.0,
                   help="watchdog floor (s): a run of n iterations gets this + 50 x n x its "
                        "expected iteration time before its waits and RCCL are aborted")
    s.add_argument("--bind-cpus", action="store_true")
    s.add_argument("--halo-n", type=int, default=512)
    s.add_argument("--nq", type=int, default=3)
    s.add_argument("--ghost", type=int, default=3)
    s.add_argument("--neighbors", type=int, default=6)
    s.add_argument("--order", default="xyzq")
    s.add_argument("--fuse", default="choice")
    s.add_argument("--transport", default="auto")
    s.add_argument("--relay", default="auto", choices=["auto", "off", "force"],
                   help="halo, 2x2x2 ranks: route a share of every face through the corner peer")
    s.add_argument("--relay-fracs", default="0.15,0.2,0.25",
                   help="relayed shares offered to the search (comma-separated)")
    s.add_argument("--hostsplit", default="auto", choices=["auto", "off", "force"],
                   help="halo, ipc receive buffers: send a share of every face through node "
                        "shared host memory over the GPUs' PCIe links, beside xGMI")
    s.add_argument("--hostsplit-fracs", default="0.1,0.2,0.3,0.4",
                   help="host shares offered to the search (comma-separated)")
    s.add_argument("--hostsplit-chunks", type=int, default=1,
                   help="host share pipelined in this many chunks (1: store, then DMA)")
    s.add_argument("--wide-puts", default="auto", choices=["auto", "on", "off"],
                   help="halo, ipc: offer kernel puts with --wide-put-blocks workgroups per box "
                        "beside the default (auto: when peers sit on other devices)")
    s.add_argument("--wide-put-blocks", type=int, default=256,
                   help="workgroups per box of the wide put")
    s.add_argument("--ipc-grid", default="auto", choices=["auto", "0", "1"],
                   help="halo, ipc: puts into the peer's grid (1) or receive buffers (0); auto: "
                        "TZ_IPC_GRID if set, else the grid below 2 GiB")
    s.add_argument("--copy-puts", default="on", choices=["on", "off"],
                   help="halo, ipc receive buffers: offer copy-engine puts")
    s.add_argument("--copy-engines", type=int, default=1,
                   help="halo: copy-engine puts of one group over this many streams")
    s.add_argument("--move-pairs", default="on", choices=["on", "off"],
                   help="halo, xyzq: x self-wrap moves as row pairs")
    s.add_argument("--grid-memory", default="auto", choices=["auto", "coarse", "fine"],
                   help="halo: grid memory (auto: fine-grained where peers store into it, ipc "
                        "grid mode)")
    s.add_argument("--horizontal", default="on", choices=["on", "off"],
                   help="fused, one rank: offer the halo move and the SpMV as one kernel launch")
    s.add_argument("--stencil", action="store_true",
                   help="halo: add the 7-point stencil (interior beside / shell after the exchange)")
    s.add_argument("--rank-grid", default="", help="halo rank grid PXxPYxPZ (default: prime factors)")
    s.add_argument("--spmv-library", default="adaptive",
                   help="rocSPARSE CSR algorithm offered beside the hand-written kernels ('' = none)")
    s.add_argument("--spmv-m", type=int, default=150_000)
    s.add_argument("--spmv-matrix", default="",
                   help="Matrix Market file (square) instead of the random band matrix")
    s.add_argument("--spmv-form", default="choice", choices=["choice", "split", "accum"])
    s.add_argument("--spmv-transport", default="auto", choices=["auto", "rccl", "ipc"])
    s.add_argument("--spmv-distribute", default="auto", choices=["auto", "root", "local"],
                   help="several ranks: rank 0 builds / reads the matrix and sends each rank its "
                        "rows (root, the reference's setup) or every rank builds it (local)")
    s.set_defaults(fn=cmd_search)
    r = sub.add_parser("rules")
    r.add_argument("results")
    r.add_argument("--out", default="")
    r.add_argument("--plots", action="store_true", help="also write the figures (PDF)")
    r.set_defaults(fn=cmd_rules)
    e = sub.add_parser("env")
    e.add_argument("--topology", action="store_true")
    e.set_defaults(fn=cmd_env)
    k = sub.add_parser("links", help="all-pairs link matrix of the launched ranks (collective)")
    k.add_argument("--mib", type=int, default=32, help="MiB per transfer")
    k.add_argument("--iters", type=int, default=10, help="transfers per pair and engine")
    k.set_defaults(fn=cmd_links)
    u = sub.add_parser("run", help="run a schedule saved by `search --save-best` (no search)")
    u.add_argument("schedule")
    u.add_argument("--iters", type=int, default=1000)
    u.add_argument("--warmup", type=int, default=50)
    u.add_argument("--mode", default="", choices=["", "eager", "graph"],
                   help="default: the mode the schedule was searched in")
    u.add_argument("--graph-unroll", type=int, default=20)
    u.add_argument("--watchdog", type=float, default=30.0,
                   help="watchdog floor (s) per run, plus 50 x n x the expected iteration time")
    u.add_argument("--torch-model", default="on", choices=["on", "off"],
                   help="halo workloads: also check one exchange against the independent torch "
                        "model (`torch_model_check`)")
    u.set_defaults(fn=cmd_run)
    return ap


if __name__ == "__main__":
    sys.exit(main())
