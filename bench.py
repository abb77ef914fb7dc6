#!/usr/bin/env python3
"""Headline benchmark: MCTS schedule search for the 3-D 27-point halo exchange, then timing of
the best schedule found.

Metric (BASELINE.json): "best-schedule iter time (ms) + MCTS search wall-clock, 3D
halo-exchange 8 ranks". Per rank: 512^3 cells x 3 quantities (f64), ghost 3, 26 neighbours,
4 HIP streams, one process per GPU, RCCL over xGMI between ranks (weak scaling: per-GPU work is
fixed as N grows). Synthetic grid data.

Flow: (1) MCTS (FastMin) explores stream assignment x issue order x sync placement x op
implementation, every candidate compiled to a hipGraph and benchmarked on all ranks (max over
ranks), then the 4 best are re-measured interleaved; (2) the best schedule is verified for
correctness (every ghost cell checked on the device); (3) it is replayed W warm-up + K timed
iterations in eager mode and as a captured hipGraph, bracketed by barrier + device sync, max over
ranks; the faster mode is reported. `value` = ms per halo-exchange iteration (lower is better);
`search_wall_s` is reported alongside.

  python bench.py --gpus 1 --steps 100 --warmup 20
  python -m torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8 --steps 100 --warmup 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _start_deadline(seconds: float) -> None:
    """A hung collective (a rank that died during communicator setup, a deadlocked transfer)
    must not hold the node forever: past the deadline every rank exits with status 4."""
    if seconds <= 0:
        return
    import threading

    def fire():
        print(f"bench.py: deadline of {seconds:.0f} s exceeded; aborting", file=sys.stderr,
              flush=True)
        os._exit(4)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def link_probe(tz, halo, ctrl, iters, rccl=False):
    """GB/s of ONE transfer over one xGMI link with each available transport (the +z face to
    the +z neighbour, every rank at once, one transfer at a time), of both z faces at once
    (`pair_GBps`: kernel puts, copy engines, or one of each), kernel puts over the x and y face
    links as well (`put_GBps_by_axis`, where those faces are remote), and the time the exchange's
    busiest link (the peer receiving the most bytes) would take at the best of those rates. An
    exchange runs several transfers per link at once (several streams, copy engines), so it can
    beat that time; on loopback ranks (one GPU) the rates say nothing about xGMI."""
    dirs = [halo.dir(i) for i in range(halo.ndirs())]
    if (0, 0, 1) not in dirs:
        return None
    i = dirs.index((0, 0, 1))
    if halo.is_direct(i):
        return None
    face = 8.0 * halo.box_elems(i)
    rates = {}
    for via in ("put", "sdma") + (("rccl",) if rccl else ()):
        try:
            t = halo.link_probe(i, via, iters, ctrl)
            rates[via] = face / t / 1e9
        except Exception as e:  # noqa: BLE001  (collective: every rank skips together)
            rates[via] = None
            if ctrl.rank == 0:
                print(f"bench.py: link probe {via}: {e}", file=sys.stderr)
    # both faces of the axis at once (one peer when the axis has 2 ranks): kernel puts, copy
    # engines, or one of each concurrently -- what the busiest link carries in practice
    pair = {}
    if not halo.is_direct(halo.opposite(i)):
        for how in ("put", "sdma", "mixed"):
            try:
                t = halo.link_probe(i, "pair_" + how, iters, ctrl)
                pair[how] = 2.0 * face / t / 1e9
            except Exception as e:  # noqa: BLE001  (collective: every rank skips together)
                pair[how] = None
                if ctrl.rank == 0:
                    print(f"bench.py: link probe pair_{how}: {e}", file=sys.stderr)
    # the other axes' face links too (kernel puts): are the links of one node alike?
    by_axis = {"z": rates.get("put")}
    for name, d in (("x", (1, 0, 0)), ("y", (0, 1, 0))):
        k = dirs.index(d)
        if halo.is_direct(k):
            continue
        try:
            by_axis[name] = 8.0 * halo.box_elems(k) / halo.link_probe(k, "put", iters, ctrl) / 1e9
        except Exception as e:  # noqa: BLE001  (collective: every rank skips together)
            by_axis[name] = None
            if ctrl.rank == 0:
                print(f"bench.py: link probe put {name}: {e}", file=sys.stderr)
    per_peer = {}
    for k in range(halo.ndirs()):
        if not halo.is_direct(k):
            per_peer[halo.neighbor(k)] = per_peer.get(halo.neighbor(k), 0.0) + 8.0 * halo.box_elems(k)
    busiest = max(per_peer.values()) if per_peer else 0.0
    best = max([r for r in list(rates.values()) + list(pair.values()) if r], default=None)
    return {"face_MB": face / 1e6, "GBps": rates, "pair_GBps": pair, "put_GBps_by_axis": by_axis,
            "busiest_link_MB": busiest / 1e6,
            "busiest_link_at_probe_rate_ms": (busiest / (best * 1e9) * 1e3) if best else None}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cells", "--n", dest="n", type=int, default=512,
                    help="interior cells per axis per rank (use --cells under torchrun: it "
                         "swallows --n as an abbreviation of its own options)")
    ap.add_argument("--neighbors", type=int, default=26)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--order", default="qxyz", choices=["xyzq", "qxyz"],
                    help="grid storage order (reference halo driver: xyzq)")
    ap.add_argument("--transport", default="auto",
                    choices=["auto", "direct", "copy", "rccl", "ipc"],
                    help="auto: direct (pack-free) moves for self-neighbours, RCCL between "
                         "ranks; ipc: pack-free puts into IPC-mapped peer grids")
    ap.add_argument("--rank-grid", default="",
                    help="PXxPYxPZ rank grid (default: the reference rule, prime factors to the "
                         "smallest dimension: 8 -> 2x2x2). Per-rank work is fixed either way; "
                         "slabs (1x1xN) send 2 instead of 6 faces per rank")
    ap.add_argument("--stencil", action="store_true",
                    help="exchange + 7-point stencil per iteration (not the BASELINE metric): the "
                         "search may update the interior while ghosts are in flight")
    ap.add_argument("--relay", default="auto", choices=["auto", "off", "force"],
                    help="2x2x2 ranks (8 GPUs): offer relay routing of a share of every face "
                         "through the corner peer's idle links (auto), never, or only it")
    ap.add_argument("--fuse", default="choice",
                    help="choice: the search picks per-direction or fused ops per group")
    ap.add_argument("--mcts-iters", type=int, default=0,
                    help="MCTS iterations (0: 40 on one rank; 120 on several, where the tree "
                         "adds transport alternatives: RCCL, IPC kernel / SDMA puts, relays)")
    ap.add_argument("--search-budget-s", type=float, default=120.0)
    # per candidate: 6 measurements of >= 2 ms each; the 4 best are re-measured interleaved
    # (--rerank) before the final timing. 20 x 4 ms, 10 x 3 ms, 8 x 2 ms and 5 x 1.5 ms all find
    # the same best schedule; 6 x 2 ms halves the search wall-clock of 10 x 3 ms
    # (profiles/r1_search_len/)
    ap.add_argument("--bench-iters", type=int, default=6)
    ap.add_argument("--target-secs", type=float, default=0.002)
    ap.add_argument("--race-ratio", type=float, default=1.25,
                    help="stop measuring a candidate once race-min measurements are all slower "
                         "than this times the best so far (0 = measure every candidate fully)")
    # settling: a candidate whose first 4 measurements agree within 3 % is measured enough
    # (search 0.62-0.68 -> 0.53-0.57 s, same best schedule and timed value, profiles/r2_settle/)
    ap.add_argument("--settle-ratio", type=float, default=0.03,
                    help="stop measuring a candidate once its first 4 measurements agree within "
                         "this ratio (0 = off)")
    ap.add_argument("--strategy", default="FastMin")
    ap.add_argument("--search-mode", default="graph", choices=["eager", "graph"],
                    help="benchmark candidates eagerly or compiled to hipGraphs (default: graph, "
                         "the way the final number is measured; eager rankings can mislead, "
                         "profiles/r1_bench_loopback/)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph-unroll", type=int, default=20,
                    help="iterations per hipGraph launch when timing the graph-compiled schedule")
    ap.add_argument("--search-graph-unroll", type=int, default=10,
                    help="iterations per hipGraph launch while benchmarking candidates (shorter "
                         "graphs compile faster; the ranking does not depend on it)")
    ap.add_argument("--rerank", type=int, default=4,
                    help="re-measure the K best distinct candidates interleaved, compiled as "
                         "hipGraphs, and keep the fastest (0: trust the search's ranking)")
    ap.add_argument("--csv", default="", help="write the search results CSV here (rank 0)")
    ap.add_argument("--save-best", default="",
                    help="write the best schedule and this workload's options (rank 0) in the "
                         "format `python -m tenzing_amd run` and `tz-search --run` take")
    ap.add_argument("--link-probe-iters", type=int, default=20,
                    help="several ranks: after the timing, measure what one xGMI link carries "
                         "per transport (one face to one peer at a time; 0 = skip)")
    ap.add_argument("--link-probe-rccl", action="store_true",
                    help="also probe RCCL (off by default: an RCCL transfer has no device-side "
                         "timeout, and a hang there would cost the whole run's output)")
    ap.add_argument("--deadline-s", type=float, default=1500.0,
                    help="abort (exit 4) if the whole run takes longer (hung collective)")
    args = ap.parse_args()
    _start_deadline(args.deadline_s)

    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.parallel import init

    ctrl, device = init()
    rank, world = ctrl.rank, ctrl.size
    if device < 0:
        print("bench.py: no GPU visible", file=sys.stderr)
        return 2
    if world != args.gpus and rank == 0:
        print(f"bench.py: warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    t_setup = time.time()
    grid = tuple(int(v) for v in args.rank_grid.lower().split("x")) if args.rank_grid else ()
    if grid and (len(grid) != 3 or grid[0] * grid[1] * grid[2] != world):
        print(f"bench.py: --rank-grid {args.rank_grid} does not factor {world} ranks",
              file=sys.stderr)
        return 2
    cfg = HaloConfig(n=args.n, neighbors=args.neighbors, fuse=args.fuse, order=args.order,
                     transport=args.transport, rank_grid=grid, stencil=args.stencil,
                     relay=args.relay)
    halo, graph = build_halo(cfg, ctrl, device)
    mode = tz.ExecMode.Graph if args.search_mode == "graph" else tz.ExecMode.Eager
    rt = tz.HipRuntime(device=device, n_streams=args.streams, mode=mode, watchdog_s=120.0,
                       graph_unroll=args.search_graph_unroll if args.search_mode == "graph" else 1)
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    setup_s = time.time() - t_setup

    opts = tz.MctsOpts()
    opts.n_iters = args.mcts_iters if args.mcts_iters > 0 else (40 if world == 1 else 120)
    opts.time_budget_s = args.search_budget_s
    opts.strategy = args.strategy
    opts.seed = args.seed
    opts.bench = tz.BenchOpts(n_iters=args.bench_iters, max_retries=3, target_secs=args.target_secs,
                              race_ratio=args.race_ratio, settle_ratio=args.settle_ratio)
    platform = tz.Platform(n_streams=args.streams)
    # candidates that cannot be compiled to a hipGraph are skipped by the search (every rank
    # agrees: preparation is collective); if none could be measured, search eagerly instead
    res = tz.mcts_explore(graph, platform, bench, ctrl, opts)
    measured = float(len(res.sims)) if rank == 0 else 1.0
    if mode == tz.ExecMode.Graph and ctrl.allreduce_max([0.0 if measured else 1.0])[0] > 0:
        print(f"bench.py: rank {rank}: no candidate could run as a hipGraph "
              f"({res.failed} skipped); searching eagerly", file=sys.stderr)
        mode = tz.ExecMode.Eager
        rt.set_mode(mode)
        rt.set_graph_unroll(1)
        res = tz.mcts_explore(graph, platform, bench, ctrl, opts)
    search_wall = res.wall_s

    # the K best distinct candidates (by the search's pct10) -> every rank
    payload = ""
    if rank == 0:
        order = sorted(range(len(res.sims)), key=lambda i: res.sims[i].res.pct10)
        top, keys = [], set()
        for i in order:
            k = res.sims[i].seq.canonical_key()
            if k not in keys:
                keys.add(k)
                top.append(i)
            if len(top) >= max(1, args.rerank):
                break
        payload = json.dumps({"seqs": [res.sims[i].seq.json() for i in top],
                              "pct10": [res.sims[i].res.pct10 for i in top],
                              "n_sims": len(res.sims), "tree": res.tree_size,
                              "failed": res.failed})
        if args.csv:
            with open(args.csv, "w") as f:
                f.write(res.dump_csv())
    payload = json.loads(ctrl.bcast(payload, 0).decode())
    index = tz.OpIndex(graph)
    cands = [index.sequence_from_json(j) for j in payload["seqs"]]
    best, best_pct10 = cands[0], payload["pct10"][0]
    rerank = None
    if args.rerank > 1 and len(cands) > 1:
        # the search measured candidates one after another (eagerly by default); the final
        # number is a compiled-graph replay, so re-rank the finalists the way they will run:
        # interleaved (drift spreads evenly), every candidate compiled to a hipGraph
        t_rr = time.time()
        rt.set_mode(tz.ExecMode.Graph)
        rt.set_graph_unroll(args.search_graph_unroll)
        ok = 1.0
        try:
            rr = bench.benchmark_many(cands, tz.BenchOpts(n_iters=args.bench_iters, max_retries=1,
                                                          target_secs=args.target_secs), args.seed)
        except Exception as e:  # noqa: BLE001
            print(f"bench.py: rank {rank}: re-rank failed: {e}", file=sys.stderr)
            ok, rr = 0.0, []
        if ctrl.allreduce_max([1.0 - ok])[0] == 0:
            # every rank measured the same max-over-ranks times: the same choice everywhere
            k = min(range(len(rr)), key=lambda i: rr[i].pct10)
            best = cands[k]
            rerank = {"pct10_ms": [r.pct10 * 1e3 for r in rr], "search_pct10_ms":
                      [p * 1e3 for p in payload["pct10"]], "chosen": k,
                      "wall_s": time.time() - t_rr}
        rt.set_mode(mode)
        rt.set_graph_unroll(args.search_graph_unroll if mode == tz.ExecMode.Graph else 1)

    # correctness of the winning schedule: one exchange from a fresh grid, every cell checked
    rt.set_mode(tz.ExecMode.Eager)
    halo.init_grid()
    rt.device_sync()
    ctrl.barrier()
    rt.prepare(best)
    rt.run(1)
    rt.device_sync()
    ctrl.barrier()  # peers may still be writing into my ghosts (ipc puts) until they synced
    bad = ctrl.allreduce_sum([float(halo.check_grid())])[0]
    bad += ctrl.allreduce_sum([float(halo.ipc_errors())])[0]
    if args.stencil:
        bad += ctrl.allreduce_sum([float(halo.check_stencil())])[0]

    def timed(m):
        rt.set_mode(m)
        # every rank must agree on the mode (a failed graph build on one rank would otherwise
        # leave the others blocked in a collective)
        ok = 1.0
        try:
            rt.prepare(best)
            ok = 1.0 if rt.effective_mode == m else 0.0
        except Exception as e:  # noqa: BLE001
            print(f"bench.py: rank {rank}: {m} preparation failed: {e}", file=sys.stderr)
            ok = 0.0
        if ctrl.allreduce_max([1.0 - ok])[0] > 0:
            rt.set_mode(tz.ExecMode.Eager)
            rt.prepare(best)
            return None, tz.ExecMode.Eager
        rt.run(args.warmup)
        rt.device_sync()
        ctrl.barrier()
        t0 = time.perf_counter()
        rt.run(args.steps)
        rt.device_sync()
        ctrl.barrier()
        dt = time.perf_counter() - t0
        return ctrl.allreduce_max([dt])[0], rt.effective_mode

    t_eager, _ = timed(tz.ExecMode.Eager)
    rt.set_graph_unroll(args.graph_unroll)
    t_graph, eff = timed(tz.ExecMode.Graph)
    # and again after every timed exchange (ghosts of an unchanged interior must still be
    # exact): catches anything that goes wrong only in later iterations, e.g. a receiver
    # reading lines its caches kept from the previous exchange
    rt.device_sync()
    ctrl.barrier()
    bad_after = ctrl.allreduce_sum([float(halo.check_grid())])[0]
    bad_after += ctrl.allreduce_sum([float(halo.ipc_errors())])[0]
    if args.stencil:
        bad_after += ctrl.allreduce_sum([float(halo.check_stencil())])[0]
    bad += bad_after
    graph_ok = t_graph is not None and eff == tz.ExecMode.Graph
    use_graph = graph_ok and t_graph < t_eager
    t = t_graph if use_graph else t_eager
    ms = t / args.steps * 1e3

    # per-link bandwidth of each transport (context for the multi-GPU number: an exchange can
    # not beat the bytes its busiest link carries divided by what one link moves)
    probe = None
    if world > 1 and args.link_probe_iters > 0:
        probe = link_probe(tz, halo, ctrl, args.link_probe_iters, args.link_probe_rccl)

    names = [o.name for o in best.ops()]
    via = [t for t, key in (("direct", "he_direct_"), ("rccl", "he_shift_"), ("ipc", "he_put_"),
                            ("sdma", "he_copyput_"), ("relay", "he_rl"))
           if any(n.startswith(key) for n in names)]
    if rank == 0:
        bytes_total = halo.exchange_bytes() * world
        out = {
            "metric": ("best-schedule iter time (ms) + MCTS search wall-clock, 3D halo-exchange 8 ranks"
                       if not args.stencil else
                       "best-schedule iter time (ms), 3D halo-exchange + 7-point stencil"),
            "value": ms,
            "unit": "ms/iter",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp64",
            "data": "synthetic",
            "config": {
                "model": f"3D {'27' if args.neighbors == 26 else '7'}-point halo-exchange "
                         f"{args.n}^3 x {cfg.nq}q ghost {cfg.ghost} per rank",
                "global_batch": world,
                "seq_len": args.n,
                "parallelism": f"{world} ranks x {args.streams} HIP streams over xGMI"
                               if world > 1 else f"1 rank x {args.streams} HIP streams",
                "streams": args.streams,
                "neighbors": args.neighbors,
                "rank_grid": list(halo.rank_grid()),
                "storage_order": args.order,
                "fuse": args.fuse,
                "strategy": args.strategy,
            },
            "search_wall_s": search_wall,
            "mcts_candidates": payload["n_sims"],
            "mcts_skipped": payload["failed"],
            "mcts_raced": bench.raced,
            "mcts_tree_nodes": payload["tree"],
            "search_mode": "hipgraph" if mode == tz.ExecMode.Graph else "eager",
            "search_best_pct10_ms": best_pct10 * 1e3,
            "rerank": rerank,
            "eager_ms_per_step": t_eager / args.steps * 1e3,
            "graph_ms_per_step": (t_graph / args.steps * 1e3) if graph_ok else None,
            "timed_mode": "hipgraph" if use_graph else "eager",
            "graph_unroll": args.graph_unroll,
            "halo_bytes_per_iter_total": bytes_total,
            "halo_GBps_total": bytes_total / (ms * 1e-3) / 1e9,
            "schedule_ops": len(best),
            "schedule_sync_ops": best.count_sync_ops(),
            "verified_bad_cells": int(bad),
            "verified_bad_cells_after_timing": int(bad_after),
            "setup_s": setup_s,
            "transport": halo.transport(),
            "schedule_transport": "+".join(via),
            "stencil_mode": (("split" if "st_interior" in names else "after")
                             if args.stencil else None),
            "ipc_mode": halo.ipc_mode() or None,
            "relay_offered": halo.uses_relay(),
            "link_probe": probe,
        }
        print(json.dumps(out), flush=True)
        if args.save_best:
            doc = {"tenzing_amd": tz.__version__, "ranks": world,
                   "mode": "graph" if use_graph else "eager", "pct10_ms": ms,
                   "args": {"workload": "halo", "streams": args.streams, "halo_n": args.n,
                            "nq": cfg.nq, "ghost": cfg.ghost, "neighbors": args.neighbors,
                            "order": args.order, "fuse": args.fuse, "transport": args.transport,
                            "relay": args.relay,
                            "relay_fracs": ",".join(str(f) for f in cfg.relay_fracs),
                            "stencil": bool(args.stencil), "rank_grid": args.rank_grid},
                   "schedule": json.loads(best.json(True))}
            with open(args.save_best, "w") as f:
                json.dump(doc, f, indent=1)
    return 0 if bad == 0 else 3


if __name__ == "__main__":
    sys.exit(main())
