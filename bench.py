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

import os
import time

# the deadline counts from here (before the first, slow, import of torch); ranks this script
# started itself count from their launcher's start
T_START = float(os.environ.get("TZ_BENCH_T0", time.time()))

import argparse  # noqa: E402
import json  # noqa: E402
import signal  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

# what a launcher exports: torchrun / torch.distributed.run, MPICH hydra / PMI, MVAPICH, Open MPI,
# Slurm srun (PMIx)
_LAUNCHER_VARS = ("WORLD_SIZE", "PMI_SIZE", "PMI_RANK", "PMIX_RANK", "OMPI_COMM_WORLD_SIZE",
                  "MV2_COMM_WORLD_SIZE")
_RANK_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
              "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")


def launched_world():
    """The rank count a launcher started this process with, or None when no launcher did
    (the same rules as the native control plane: parallel/dist.py, MpiCtrl::launcher_size)."""
    e = os.environ
    if "WORLD_SIZE" in e:
        return int(e["WORLD_SIZE"])
    for v in ("OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "MV2_COMM_WORLD_SIZE"):
        if v in e:
            return int(e[v])
    if "PMIX_RANK" in e or "PMI_RANK" in e:
        return int(e.get("SLURM_NTASKS", "1"))
    return None


def _free_port() -> int:
    import socket

    # the control plane listens on MASTER_PORT + 1 (or one of the next 8): keep the pair free
    for _ in range(64):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p < 65000:
            return p
    return 29500


def spawn_ranks(n: int, argv, deadline_s: float) -> int:
    """Start `n` fresh rank processes of this script (one per GPU, RANK / WORLD_SIZE /
    LOCAL_RANK / MASTER_* set, rendezvous over 127.0.0.1) and relay rank 0's result line.

    Runs before anything imports torch or tenzing_amd: this process never touches the GPU and
    never execs. Exit status: 0 when every rank exited 0; otherwise the first failing rank's
    status (124 when the ranks outlived the deadline and were killed). A run whose rank 0 printed
    no line gets a partial one from here, so the failure still says what happened."""
    port = _free_port()
    base = {k: v for k, v in os.environ.items() if k not in _RANK_VARS + _LAUNCHER_VARS}
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), TZ_BENCH_T0=repr(T_START), TZ_BENCH_SPAWNED="1")
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        # a session of its own per rank: the whole process group is signalled on the way out
        procs.append(subprocess.Popen(
            [sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
            stdout=subprocess.PIPE if r == 0 else sys.stderr, start_new_session=True, text=True))

    def kill(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def on_signal(sig, _frame):
        kill(sig)
        raise SystemExit(128 + sig)

    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, on_signal)
    # rank 0's stdout, line by line on a thread: progress passes through as it comes, and the
    # JSON line goes to stdout exactly once
    import threading

    lines = []

    def pump():
        for line in procs[0].stdout:
            if line.startswith("{"):
                lines.append(line.strip())
            else:
                sys.stderr.write(line)
                sys.stderr.flush()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    # the ranks own their deadline (they print a partial line at it); this bound is the
    # backstop for ranks that cannot even reach theirs
    limit = (T_START + deadline_s + 30.0) if deadline_s > 0 else None
    failed_at = None
    rc = 0
    while any(p.poll() is None for p in procs):
        now = time.time()
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad and failed_at is None:
            failed_at = now  # peers of a failed rank get a grace period to report, then go
        if (failed_at is not None and now - failed_at > 30.0) or (limit and now > limit):
            rc = rc or (bad[0] if bad else 124)
            kill(signal.SIGTERM)
            time.sleep(5.0)
            kill(signal.SIGKILL)
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
    t.join(timeout=10.0)
    codes = [p.returncode for p in procs]
    rc = rc or next((c for c in codes if c != 0), 0)
    if lines:
        print(lines[-1], flush=True)
    elif rc != 0:
        print(json.dumps({"metric": _METRIC, "value": None, "n_gpus": n, "partial": True,
                          "phase": "launch", "error": f"rank exit codes {codes}",
                          "launcher": "bench.py"}), flush=True)
    if rc != 0:
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr, flush=True)
    return rc if rc > 0 else (128 - rc) if rc < 0 else 0


_METRIC = "best-schedule iter time (ms) + MCTS search wall-clock, 3D halo-exchange 8 ranks"


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
    for via in ("put", "put_wide", "sdma", "memcpy") + (("rccl",) if rccl else ()):
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
        for how in ("put", "put_wide", "sdma", "mixed"):
            try:
                t = halo.link_probe(i, "pair_" + how, iters, ctrl)
                pair[how] = 2.0 * face / t / 1e9
            except Exception as e:  # noqa: BLE001  (collective: every rank skips together)
                pair[how] = None
                if ctrl.rank == 0:
                    print(f"bench.py: link probe pair_{how}: {e}", file=sys.stderr)
    # the kernel put's width over the same link: workgroups per box (the default put runs 64,
    # the wide put 256); on a node this says which width fills an xGMI link
    by_cap = {}
    for cap in (16, 64, 256, 1024):
        try:
            by_cap[str(cap)] = face / halo.link_probe(i, f"put_cap{cap}", iters, ctrl) / 1e9
        except Exception as e:  # noqa: BLE001  (collective: every rank skips together)
            by_cap[str(cap)] = None
            if ctrl.rank == 0:
                print(f"bench.py: link probe put_cap{cap}: {e}", file=sys.stderr)
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
            "put_GBps_by_blocks_per_box": by_cap,
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
                    choices=["auto", "direct", "copy", "rccl", "ipc", "host"],
                    help="auto: direct (pack-free) moves for self-neighbours; between ranks the "
                         "search chooses among RCCL, IPC kernel puts, copy-engine puts and "
                         "relays, whichever passed its preflight (the host-staged transport if "
                         "none did); host: the host-staged transport only")
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
    ap.add_argument("--hostsplit", default="auto", choices=["auto", "off", "force"],
                    help="several ranks, ipc receive buffers: offer sending a share of every "
                         "face through node shared host memory over each GPU's PCIe link, "
                         "beside xGMI (auto), never, or only it")
    ap.add_argument("--hostsplit-chunks", type=int, default=1,
                    help="host share pipelined in this many chunks (1: all stores, then the DMA)")
    ap.add_argument("--wide-puts", default="auto", choices=["auto", "on", "off"],
                    help="several ranks, ipc: offer kernel puts with --wide-put-blocks "
                         "workgroups per box beside the default 64 (auto: when the peers sit "
                         "on other devices, i.e. puts cross xGMI)")
    ap.add_argument("--wide-put-blocks", type=int, default=256,
                    help="workgroups per box of the wide put")
    ap.add_argument("--copy-puts", default="on", choices=["on", "off"],
                    help="several ranks, ipc receive buffers: offer copy-engine puts")
    ap.add_argument("--fuse", default="choice",
                    help="choice: the search picks per-direction or fused ops per group")
    ap.add_argument("--mcts-iters", type=int, default=0,
                    help="MCTS iterations (0: 40 on one rank; 120 on several, where the tree "
                         "adds transport alternatives: RCCL, IPC kernel / copy-engine puts, relays)")
    ap.add_argument("--search-budget-s", type=float, default=120.0)
    # per candidate: 6 measurements of >= 2 ms each; the 4 best are re-measured interleaved
    # (--rerank) before the final timing. 20 x 4 ms, 10 x 3 ms, 8 x 2 ms and 5 x 1.5 ms all find
    # the same best schedule; 6 x 2 ms halves the search wall-clock of 10 x 3 ms
    # (profiles/archive/r1_search_len/)
    ap.add_argument("--bench-iters", type=int, default=6)
    ap.add_argument("--target-secs", type=float, default=0.002)
    ap.add_argument("--race-ratio", type=float, default=1.25,
                    help="stop measuring a candidate once race-min measurements are all slower "
                         "than this times the best so far (0 = measure every candidate fully)")
    # settling: a candidate whose first 4 measurements agree within 3 % is measured enough
    # (search 0.62-0.68 -> 0.53-0.57 s, same best schedule and timed value, profiles/archive/r2_settle/)
    ap.add_argument("--settle-ratio", type=float, default=0.03,
                    help="stop measuring a candidate once its first 4 measurements agree within "
                         "this ratio (0 = off)")
    ap.add_argument("--strategy", default="FastMin")
    ap.add_argument("--search-mode", default="graph", choices=["eager", "graph"],
                    help="benchmark candidates eagerly or compiled to hipGraphs (default: graph, "
                         "the way the final number is measured; eager rankings can mislead, "
                         "profiles/archive/r1_bench_loopback/)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seed-transports", type=int, default=1,
                    help="several ranks: measure one fused schedule per remote transport before "
                         "the search (each transport is then measured at least once; 0 = off)")
    ap.add_argument("--sim-seeds", type=int, default=2,
                    help="several ranks: also seed the search with the K best schedules of a "
                         "short hardware-free search under the link-aware cost model (0 = off)")
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
    ap.add_argument("--deadline-s", type=float, default=540.0,
                    help="wall-clock limit of the whole run, from process start (below the "
                         "driver's 600 s): past it rank 0 prints its best result so far as the "
                         "normal JSON line with \"partial\": true and every rank exits with "
                         "status 5 (0 = no limit)")
    ap.add_argument("--watchdog-s", type=float, default=10.0,
                    help="watchdog floor per run of a candidate: a run of n iterations gets "
                         "this + --watchdog-k x n x its expected iteration time, then its device "
                         "waits and RCCL communicators are aborted and the candidate is skipped")
    ap.add_argument("--watchdog-k", type=float, default=50.0)
    ap.add_argument("--ghost-align", type=int, default=-2,
                    help="x ghost runs aligned to 16 (line) / 8 (sector) elements, 0 = interior "
                         "rows sector-aligned, -1 = x=0 at the pitched row start (reference), "
                         "-2 = auto (16, line-aligned, in both orders)")
    ap.add_argument("--torch-model", default="on", choices=["on", "off"],
                    help="after the headline: one more exchange of the timed schedule from a "
                         "hashed field, checked against an independent torch model "
                         "(`torch_model_check`)")
    ap.add_argument("--subrecords", default="auto", choices=["auto", "on", "off"],
                    help="after the headline: BASELINE configs 2 (SpMV, band m / ranks) and 5 "
                         "(SpMV + halo), each searched briefly over this run's transports, "
                         "verified and timed, and on one rank also the reference's XYZQ layout "
                         "and the move's roof (auto = on: every rank count; off: none)")
    ap.add_argument("--post-budget-s", type=float, default=150.0,
                    help="once the headline is final: wall-clock budget of the sub-records and "
                         "diagnostics after it; past it the complete line is printed and the run "
                         "exits 0")
    ap.add_argument("--link-matrix-wait-s", type=float, default=20.0,
                    help="several ranks: the all-pairs link matrix gives up on a transfer that "
                         "has not completed within this (the record then says so)")
    ap.add_argument("--branch-probe", default="on", choices=["on", "off"],
                    help="probe whether 3 independent branches of a hipGraph run at once with "
                         "this runtime's stream padding (else try other paddings); recorded")
    args = ap.parse_args()

    # one process per GPU: a launcher (torchrun, mpiexec, srun) may have started the ranks;
    # otherwise this process starts them itself, before anything touches the GPU
    launched = launched_world()
    if launched is None and args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:], args.deadline_s)
    if (launched or 1) != args.gpus:
        print(f"bench.py: --gpus {args.gpus}, but the launcher started {launched} rank(s): "
              "a scaling point must measure the rank count it names", file=sys.stderr)
        return 2

    # one node (every rank local): RCCL's bootstrap over the loopback interface, which always
    # exists, instead of whichever interface it would pick (its data moves over xGMI either way)
    if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and "NCCL_SOCKET_IFNAME" not in os.environ
            and os.environ.get("LOCAL_WORLD_SIZE", "") == os.environ.get("WORLD_SIZE")):
        os.environ["NCCL_SOCKET_IFNAME"] = "lo"

    import tenzing_amd as tz
    from tenzing_amd.utils.benchkit import remote_via, schedule_via
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.parallel import init
    from tenzing_amd.utils.env import runtime_libraries

    elapsed = time.time() - T_START
    deadline = (tz.RunDeadline(max(1.0, args.deadline_s - elapsed), 5)
                if args.deadline_s > 0 else None)

    ctrl, device = init()
    rank, world = ctrl.rank, ctrl.size
    if device < 0:
        print(f"bench.py: rank {rank}: no GPU visible", file=sys.stderr)
        return 2
    if world != args.gpus:
        print(f"bench.py: rank {rank}: --gpus {args.gpus} but {world} ranks joined", file=sys.stderr)
        return 2
    cpus = []
    if world > 1:
        # one process per GPU: keep each rank's host threads on the CPUs next to its GPU
        from tenzing_amd.utils.env import bind_local_cpus
        try:
            cpus = bind_local_cpus(device)
        except Exception as e:  # noqa: BLE001
            print(f"bench.py: rank {rank}: CPU binding failed: {e}", file=sys.stderr)

    grid = tuple(int(v) for v in args.rank_grid.lower().split("x")) if args.rank_grid else ()
    if grid and (len(grid) != 3 or grid[0] * grid[1] * grid[2] != world):
        print(f"bench.py: --rank-grid {args.rank_grid} does not factor {world} ranks",
              file=sys.stderr)
        return 2
    cfg = HaloConfig(n=args.n, neighbors=args.neighbors, fuse=args.fuse, order=args.order,
                     transport=args.transport, rank_grid=grid, stencil=args.stencil,
                     relay=args.relay, hostsplit=args.hostsplit,
                     hostsplit_chunks=args.hostsplit_chunks, wide_puts=args.wide_puts,
                     wide_put_blocks=args.wide_put_blocks, ghost_align=args.ghost_align,
                     copy_puts=args.copy_puts == "on")

    # the JSON line: every field known up front, so that the deadline can print it partially
    out = {
        "metric": (_METRIC if not args.stencil else
                   "best-schedule iter time (ms), 3D halo-exchange + 7-point stencil"),
        "value": None,
        "unit": "ms/iter",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
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
            "rank_grid": None,
            "storage_order": args.order,
            "fuse": args.fuse,
            "strategy": args.strategy,
        },
        "partial": True,
        "phase": "setup",
        "deadline_s": args.deadline_s,
        # who started the ranks: this script itself (no launcher in the environment), torchrun,
        # or an MPI launcher
        "launcher": ("bench.py" if os.environ.get("TZ_BENCH_SPAWNED") == "1" else
                     "mpi" if "WORLD_SIZE" not in os.environ and world > 1 else
                     "torchrun" if world > 1 else None),
    }

    _STATE.update(out=out, rank=rank, deadline=deadline)

    def report(**kw):
        """rank 0: what the deadline prints if the run cannot finish (the best so far)"""
        out.update(kw)
        if deadline is not None and rank == 0:
            out["elapsed_s"] = round(time.time() - T_START, 1)
            deadline.set_report(json.dumps(out))

    report()
    t_setup = time.time()
    halo, graph = build_halo(cfg, ctrl, device)
    out["config"]["rank_grid"] = list(halo.rank_grid())
    mode = tz.ExecMode.Graph if args.search_mode == "graph" else tz.ExecMode.Eager

    def make_rt(pad=None, n_streams=args.streams):
        return tz.HipRuntime(device=device, n_streams=n_streams, mode=mode,
                             watchdog_s=args.watchdog_s, watchdog_k=args.watchdog_k,
                             graph_unroll=args.search_graph_unroll if args.search_mode == "graph" else 1,
                             pad_streams=-1 if pad is None else pad)

    branch = None
    if args.branch_probe == "on" and args.streams >= 3:
        # the search ranks candidates as hipGraphs: check on this box that HIP's graph executor
        # runs independent branches at once with this padding (else try others)
        from tenzing_amd.utils.benchkit import branch_probe, choose_pad
        rt, branch = choose_pad(make_rt, lambda r: branch_probe(tz, r), [None, 8, 12, 4])
    else:
        rt = make_rt()
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    setup_s = time.time() - t_setup
    transports = halo.transport_report()
    # which device every peer rank sits on and whether this GPU reaches it peer-to-peer
    # (collective); rank 0's view goes into the record, the "peer_access" line into
    # transports_available
    peers = None
    if world > 1:
        from tenzing_amd.parallel.topology import peer_device_facts
        nb = [halo.neighbor(k) for k in range(halo.ndirs()) if not halo.is_direct(k)]
        peers = peer_device_facts(ctrl, device, nb, ipc_mapped=halo.ipc_peer_devices())
        transports["peer_access"] = peers["summary"]
    report(phase="search", setup_s=setup_s, transport=halo.transport(),
           transports_available=transports, rccl_nranks=halo.rccl_nranks() or None)

    platform = tz.Platform(n_streams=args.streams)
    opts = tz.MctsOpts()
    opts.n_iters = args.mcts_iters if args.mcts_iters > 0 else (40 if world == 1 else 120)
    # the search leaves time for the re-rank, the verification and the timing before the deadline
    budget = args.search_budget_s
    if deadline is not None:
        budget = max(5.0, min(budget, deadline.remaining - 90.0))
    opts.time_budget_s = budget
    opts.strategy = args.strategy
    opts.seed = args.seed
    opts.bench = tz.BenchOpts(n_iters=args.bench_iters, max_retries=3, target_secs=args.target_secs,
                              race_ratio=args.race_ratio, settle_ratio=args.settle_ratio)
    seed_alts = []
    if world > 1 and args.seed_transports:
        # one schedule per remote transport, measured before the search: every transport is
        # measured at least once however the tree's random rollouts fall (the top-level choice
        # has up to 8 alternatives, each with its own structure sub-tree)
        from tenzing_amd.search import choice_alternatives, greedy_schedule
        seeds = []
        for alt in choice_alternatives(graph, "he_remote"):
            try:
                seeds.append(greedy_schedule(
                    graph, platform, {"he_remote": alt, "*": ["allfused", "fused"]},
                    stream_for=lambda n: 1 if n.startswith("he_direct") and args.streams > 1 else 0))
                seed_alts.append(alt)
            except Exception as e:  # noqa: BLE001 (same graph on every rank: all skip alike)
                print(f"bench.py: rank {rank}: no seed schedule for {alt}: {e}", file=sys.stderr)
        sim_seeded = []
        if rank == 0 and args.sim_seeds > 0:
            # the link-aware model's own best structures (stream splits, transport mixes) as
            # extra seeds: 400 hardware-free iterations on this rank's graph, a fraction of a
            # second; a wrong model costs only these few measurements
            from tenzing_amd.parallel.linkmodel import graph_params_from_probe, link_sim_params, sim_seeds
            try:
                # the replay model's join cost as this box's branch probe measured it
                sim_params = graph_params_from_probe(link_sim_params(), branch)
                report(model_params={"graph_join_us": round(sim_params.graph_join_us, 2),
                                     "graph_wait_us": sim_params.graph_wait_us})
                for sq, us in sim_seeds(graph, platform, args.sim_seeds, 400, params=sim_params,
                                        exclude=seeds, seed=args.seed):
                    seeds.append(sq)
                    sim_seeded.append({"key": sq.canonical_key(), "model_us": round(us, 1),
                                       "transport": remote_via([o.name for o in sq.ops()])})
            except Exception as e:  # noqa: BLE001 (seeds are optional)
                print(f"bench.py: model seeds skipped: {e}", file=sys.stderr)
        if rank == 0:
            opts.seed_schedules = seeds

    best_seen = {"pct10": None, "n": 0, "said": time.time()}

    def on_result(i, sr):
        best_seen["n"] += 1
        if time.time() - best_seen["said"] > 15:
            # a heartbeat on stderr for long multi-rank searches
            best_seen["said"] = time.time()
            print(f"bench.py: search: {best_seen['n']} candidates, best pct10 "
                  f"{(best_seen['pct10'] or 0) * 1e3:.4f} ms", file=sys.stderr, flush=True)
        if best_seen["pct10"] is None or sr.res.pct10 < best_seen["pct10"]:
            best_seen["pct10"] = sr.res.pct10
            names = [o.name for o in sr.seq.ops()]
            report(value=sr.res.pct10 * 1e3, ms_per_step=sr.res.pct10 * 1e3,
                   value_source="search pct10 (the best candidate measured so far; not timed)",
                   schedule_transport="+".join(schedule_via(names)),
                   mcts_candidates=best_seen["n"])

    # candidates that cannot be compiled to a hipGraph are skipped by the search (every rank
    # agrees: preparation is collective); if none could be measured, search eagerly instead
    res = tz.mcts_explore(graph, platform, bench, ctrl, opts, on_result if rank == 0 else None)
    measured = float(len(res.sims)) if rank == 0 else 1.0
    if mode == tz.ExecMode.Graph and ctrl.allreduce_max([0.0 if measured else 1.0])[0] > 0:
        print(f"bench.py: rank {rank}: no candidate could run as a hipGraph "
              f"({res.failed} skipped); searching eagerly", file=sys.stderr)
        mode = tz.ExecMode.Eager
        rt.set_mode(mode)
        rt.set_graph_unroll(1)
        opts.time_budget_s = max(5.0, min(budget, deadline.remaining - 60.0)) if deadline else budget
        res = tz.mcts_explore(graph, platform, bench, ctrl, opts, on_result if rank == 0 else None)
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
        seeded = {}
        model = {d["key"]: d for d in (sim_seeded if world > 1 and args.seed_transports else [])}
        for s_ in res.sims:
            if s_.seeded:
                key = s_.seq.canonical_key()
                if key in model:  # a model seed: its measured time beside the model's
                    model[key]["measured_ms"] = s_.res.pct10 * 1e3
                    continue
                v = remote_via([o.name for o in s_.seq.ops()]) or "none"
                seeded[v] = s_.res.pct10 * 1e3
        model_seeded = [{k: v for k, v in d.items() if k != "key"} for d in model.values()]
        payload = json.dumps({"seqs": [res.sims[i].seq.json() for i in top],
                              "model_seeded": model_seeded,
                              "pct10": [res.sims[i].res.pct10 for i in top],
                              "n_sims": len(res.sims), "tree": res.tree_size,
                              "failed": res.failed, "seeded": seeded})
        if args.csv:
            with open(args.csv, "w") as f:
                f.write(res.dump_csv())
    payload = json.loads(ctrl.bcast(payload, 0).decode())
    if not payload["seqs"]:
        print(f"bench.py: rank {rank}: the search measured no candidate", file=sys.stderr)
        _report_failure("the search measured no candidate")
        return 4
    index = tz.OpIndex(graph)
    cands = [index.sequence_from_json(j) for j in payload["seqs"]]
    best, best_pct10 = cands[0], payload["pct10"][0]
    report(phase="rerank", search_wall_s=search_wall, mcts_candidates=payload["n_sims"],
           mcts_skipped=payload["failed"], seeded_pct10_ms=payload["seeded"] or None,
           dead_domains=list(res.dead_domains), pruned_dead=res.pruned_dead)
    rerank = None
    ranked = list(range(len(cands)))  # finalists in order of preference
    if args.rerank > 1 and len(cands) > 1:
        # the search measured candidates one after another; the final number is a compiled-graph
        # replay, so re-rank the finalists the way they will run: interleaved (drift spreads
        # evenly), every candidate compiled to a hipGraph
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
            ranked = sorted(range(len(rr)), key=lambda i: rr[i].pct10)
            k = ranked[0]
            best = cands[k]
            rerank = {"pct10_ms": [r.pct10 * 1e3 for r in rr], "search_pct10_ms":
                      [p * 1e3 for p in payload["pct10"]], "chosen": k,
                      "wall_s": time.time() - t_rr}
        rt.set_mode(mode)
        rt.set_graph_unroll(args.search_graph_unroll if mode == tz.ExecMode.Graph else 1)

    # correctness of the winning schedule: one exchange from a fresh grid, every cell checked.
    # (Device-side wait timeouts of search candidates are counted and cleared first: they belong
    # to schedules that lost, not to the one verified here.)
    search_timeouts = int(ctrl.allreduce_sum([float(halo.ipc_errors())])[0])
    report(phase="verify", search_wait_timeouts=search_timeouts)
    rt.set_mode(tz.ExecMode.Eager)

    def verify(seq, gen):
        """one exchange of `seq` from a grid of value generation `gen` (the search ran on
        generation 0, so a schedule whose transport leaves stale ghosts or buffers behind fails
        here); bad cells + wait timeouts + failed runs, summed over ranks"""
        halo.init_grid(gen=gen)
        rt.device_sync()
        ctrl.barrier()
        failed = 0.0
        try:
            rt.prepare(seq)
            rt.run(1)
            rt.device_sync()
        except Exception as e:  # noqa: BLE001 (counted below, on every rank)
            print(f"bench.py: rank {rank}: verification run failed: {e}", file=sys.stderr)
            failed = 1.0
        ctrl.barrier()  # peers may still be writing into my ghosts (ipc puts) until they synced
        b = ctrl.allreduce_sum([float(halo.check_grid())])[0]
        b += ctrl.allreduce_sum([float(halo.ipc_errors())])[0]
        if args.stencil:
            b += ctrl.allreduce_sum([float(halo.check_stencil())])[0]
        return b + ctrl.allreduce_sum([failed])[0]

    # a finalist that does not deliver (a transport that passed its preflight but fails in this
    # schedule's form) is rejected and the next one verified instead: the run reports a schedule
    # that is right rather than the fastest one that is wrong
    rejected = []
    bad = None
    reject_first = int(os.environ.get("TZ_BENCH_REJECT", "0"))  # tests: fail the first n
    for n_try, k in enumerate(ranked):
        b = verify(cands[k], 1 + n_try % 3) + (1.0 if n_try < reject_first else 0.0)
        if b == 0:
            best, bad = cands[k], 0.0
            break
        rejected.append({"rank_in_rerank": n_try, "bad": int(b),
                         "transport": remote_via([o.name for o in cands[k].ops()]) or "direct"})
        if rank == 0:
            print(f"bench.py: finalist {n_try} failed verification ({int(b)} bad); trying the "
                  "next", file=sys.stderr, flush=True)
        halo.reset_transport_state(ctrl)  # counters of a timed-out exchange restart from zero
    if bad is None:  # none verified: report the preferred one with its bad cells
        best, bad = cands[ranked[0]], float(rejected[0]["bad"])
    halo.init_grid()  # back to generation 0 for the timing and its final check
    rt.device_sync()
    ctrl.barrier()
    report(phase="timing", verified_bad_cells=int(bad), verify_rejected=rejected or None)

    from tenzing_amd.utils.benchkit import timed_replay

    def timed(m):
        return timed_replay(tz, rt, ctrl, best, m, args.steps, args.warmup)

    t_eager, _ = timed(tz.ExecMode.Eager)
    report(value=t_eager / args.steps * 1e3, ms_per_step=t_eager / args.steps * 1e3,
           value_source="eager replay of the best schedule (the hipGraph replay did not finish)",
           eager_ms_per_step=t_eager / args.steps * 1e3)
    rt.set_graph_unroll(args.graph_unroll)
    t_graph, eff = timed(tz.ExecMode.Graph)
    # what the timed hipGraph is made of (kernel / host / memcpy / event nodes per iteration):
    # e.g. whether RCCL over this node's transport adds proxy host nodes
    graph_nodes = rt.graph_node_types() if eff == tz.ExecMode.Graph else None
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
    names = [o.name for o in best.ops()]
    bytes_total = halo.exchange_bytes() * world
    n_local = sum(1 for i in range(halo.ndirs()) if halo.is_direct(i))
    out.update({
        "value": ms,
        "ms_per_step": ms,
        "value_source": "timed replay of the best schedule",
        "partial": False,
        "phase": "done",
        "search_wall_s": search_wall,
        "mcts_candidates": payload["n_sims"],
        "mcts_skipped": payload["failed"],
        "mcts_raced": bench.raced,
        "mcts_tree_nodes": payload["tree"],
        "search_mode": "hipgraph" if mode == tz.ExecMode.Graph else "eager",
        "search_best_pct10_ms": best_pct10 * 1e3,
        "seeded_pct10_ms": payload["seeded"] or None,
        "model_seeded": payload.get("model_seeded") or None,
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
        "verify_rejected": rejected or None,
        "setup_s": setup_s,
        "transport": halo.transport(),
        "transports_available": transports,
        "rccl_nranks": halo.rccl_nranks() or None,
        "schedule_transport": "+".join(schedule_via(names)),
        "transport_by_group": {"local": {"dirs": n_local, "via": "direct" if n_local else None},
                               "remote": {"dirs": halo.ndirs() - n_local,
                                          "via": remote_via(names)}},
        "dead_domains": list(res.dead_domains),
        "pruned_dead": res.pruned_dead,
        "watchdog": {"floor_s": args.watchdog_s, "k": args.watchdog_k,
                     "fired": rt.watchdog_fired},
        "search_wait_timeouts": search_timeouts,
        "stencil_mode": (("split" if "st_interior" in names else "after")
                         if args.stencil else None),
        "ipc_mode": halo.ipc_mode() or None,
        "relay_offered": halo.uses_relay(),
        "hostsplit_offered": halo.uses_hostsplit(),
        "hostsplit_chunks": cfg.hostsplit_chunks if halo.uses_hostsplit() else None,
        "wide_puts_offered": halo.uses_wide_puts(),
        "cpus_bound": len(cpus) or None,
        "rccl_socket_ifname": os.environ.get("NCCL_SOCKET_IFNAME") if world > 1 else None,
        "peer_devices": peers,
        "runtime": runtime_libraries(),
        "graph_capture": tz._tz.graph_capture_info(),
        "graph_branch_probe": branch,
        "pad_streams": rt.pad_streams,
        "timed_graph_node_types": graph_nodes,
    })
    # The headline is final. Everything after it is optional and bounded: from here the deadline
    # prints this (complete) line and exits 0 if the sub-records or diagnostics do not finish
    # within --post-budget-s, so a stall there (e.g. the first cross-device transfer of a link
    # probe) cannot turn a finished measurement into a partial one.
    post = {"budget_s": args.post_budget_s, "done": [], "running": None}
    out["post_timing"] = post
    # the best schedule, saved before anything optional runs
    if rank == 0 and args.save_best:
        doc = {"tenzing_amd": tz.__version__, "ranks": world,
               "mode": "graph" if use_graph else "eager", "pct10_ms": ms,
               "args": {"workload": "halo", "streams": args.streams, "halo_n": args.n,
                        "nq": cfg.nq, "ghost": cfg.ghost, "neighbors": args.neighbors,
                        "order": args.order, "fuse": args.fuse, "transport": args.transport,
                        "relay": args.relay,
                        "relay_fracs": ",".join(str(f) for f in cfg.relay_fracs),
                        "hostsplit": args.hostsplit,
                        "hostsplit_fracs": ",".join(str(f) for f in cfg.hostsplit_fracs),
                        "hostsplit_chunks": cfg.hostsplit_chunks,
                        "wide_puts": args.wide_puts, "wide_put_blocks": args.wide_put_blocks,
                        "copy_puts": args.copy_puts,
                        "ipc_grid": {"grid": "1", "buffers": "0"}.get(halo.ipc_mode(), "auto"),
                        "stencil": bool(args.stencil), "rank_grid": args.rank_grid},
               "schedule": json.loads(best.json(True))}
        with open(args.save_best, "w") as f:
            json.dump(doc, f, indent=1)

    def post_phase(name):
        post["running"] = name
        report()
        stall = os.environ.get("TZ_BENCH_STALL", "")  # tests: hang in this phase
        if stall == name:
            time.sleep(1e6)

    def post_done(name, **kw):
        post["done"].append(name)
        post["running"] = None
        report(**kw)

    if deadline is not None:
        report()
        deadline.tighten(max(5.0, min(args.post_budget_s, deadline.remaining - 10.0)),
                         0 if bad == 0 else 3)

    stuck = False
    if args.torch_model == "on":
        # the timed schedule once more against a model that shares no code with the exchange
        # (tenzing_amd/utils/halo_ref.py): every rank loads its block of a hashed global field,
        # runs one exchange and compares its whole padded block with torch's periodic model
        post_phase("torch_model")
        post_done("torch_model", torch_model_check=_torch_model_check(tz, rt, ctrl, halo, device))
    # per-link bandwidth of each transport (context for the multi-GPU number: an exchange can
    # not beat the bytes its busiest link carries divided by what one link moves)
    if world > 1 and args.link_probe_iters > 0:
        post_phase("link_probe")
        probe = link_probe(tz, halo, ctrl, args.link_probe_iters, args.link_probe_rccl)
        post_done("link_probe", link_probe=probe)
        # every ordered pair of ranks (not only the halo's neighbours), every rank sending at
        # once: the fabric the search ran on, e.g. whether all pairs are one xGMI hop
        post_phase("link_matrix")
        try:
            matrix = tz._tz.link_matrix(ctrl, 32 << 20, 10, args.link_matrix_wait_s)
            stuck = bool(matrix.get("stuck"))
            from tenzing_amd.parallel.topology import matrix_summary
            matrix["summary"] = {k: matrix_summary(matrix[k + "_GBps"]) for k in ("put", "sdma")}
        except Exception as e:  # noqa: BLE001
            matrix = {"why": str(e)}
        post_done("link_matrix", link_matrix=matrix)
        if halo.uses_relay():
            # the relayed share the link model balances with, at equal link rates (offered to
            # the search) and at this run's own measured rates (for the record)
            from tenzing_amd.parallel.linkmodel import relay_share, relay_share_from_record
            f_meas = relay_share_from_record({"config": {"rank_grid": list(halo.rank_grid())},
                                              "link_matrix": matrix})
            report(relay_shares={"offered": list(cfg.relay_fracs), "f_star_equal_rates": relay_share(),
                                 "f_star_link_matrix": round(f_meas, 3) if f_meas else None})
    if rank == 0 and world > 1:
        post_phase("topology")
        from tenzing_amd.utils.env import xgmi_topology_summary
        post_done("topology", xgmi_topology=xgmi_topology_summary())
        if args.link_probe_iters > 0 and not stuck:
            # the link-aware model, calibrated on this run's own link rates, against this run's
            # measured per-transport seeds (host-only, rank 0, under a second)
            post_phase("model_check")
            try:
                from tenzing_amd.parallel.linkmodel import model_report
                mc = model_report(out)
                val = {k: mc[k] for k in ("seeds", "spearman", "best_by_model", "best_measured")}
            except Exception as e:  # noqa: BLE001 (a diagnostic)
                val = {"error": f"{type(e).__name__}: {e}"}
            post_done("model_check", model_check=val)

    subrecords = args.subrecords in ("on", "auto")
    if subrecords and not stuck and world == 1 and halo.uses_direct():
        # the headline's move kernel against a kernel that touches exactly the same lines
        post_phase("move_roof")
        try:
            val = halo.move_roof(20)
        except Exception as e:  # noqa: BLE001
            val = {"error": f"{type(e).__name__}: {e}"}
        post_done("move_roof", move_roof=val)
    if subrecords and not stuck:
        # the other BASELINE configs (and, on one rank, the reference driver's layout), each in
        # this same run; at N > 1 they run over the same transports as the headline
        ctrl.barrier()  # no peer still reads or writes this rank's headline buffers
        del bench
        rt = None  # the headline's runtime and streams go before the sub-records' are made
        halo = None
        subs = (("reference_layout", _reference_layout),) if world == 1 else ()
        for name, fn in subs + (("baseline_configs", _baseline_configs),):
            post_phase(name)
            try:
                val = fn(tz, args, ctrl, device, branch)
            except Exception as e:  # noqa: BLE001 (a sub-record never costs the headline)
                val = {"error": f"{type(e).__name__}: {e}"}
                print(f"bench.py: rank {rank}: {name}: {val['error']}", file=sys.stderr, flush=True)
            out[name] = val
            post_done(name)

    out["elapsed_s"] = round(time.time() - T_START, 1)
    if rank == 0:
        if deadline is not None:
            deadline.cancel()
        print(json.dumps(out), flush=True)
    elif deadline is not None:
        deadline.cancel()
    if stuck:
        # a diagnostic transfer never completed: the device may never drain, so the runtime's
        # teardown at exit could hang; the result is out, leave without it
        sys.stdout.flush()
        os._exit(0 if bad == 0 else 3)
    return 0 if bad == 0 else 3


def _torch_model_check(tz, rt, ctrl, halo, device):
    """one exchange of the prepared (timed) schedule from a hashed field, every cell of every
    rank's padded block compared with tenzing_amd.utils.halo_ref's model; bad cells summed over
    ranks by ghost class (interior, face, edge, corner). The grid is re-initialized afterwards."""
    t0 = time.time()
    try:
        from tenzing_amd.utils.halo_ref import check_prepared

        val = check_prepared(halo, rt, ctrl, device)
    except Exception as e:  # noqa: BLE001 (a diagnostic after the headline)
        val = {"error": f"{type(e).__name__}: {e}"}
    try:
        halo.init_grid()
        rt.device_sync()
    except Exception as e:  # noqa: BLE001
        val["restore_error"] = f"{type(e).__name__}: {e}"
    val["s"] = round(time.time() - t0, 2)
    return val


def _sub_runtime(tz, args, device, branch, n_streams):
    """a runtime for a sub-record: graph-mode search, the headline's watchdog and padding"""
    pad = branch["pad_streams"] if branch and branch.get("pad_streams") else -1
    return tz.HipRuntime(device=device, n_streams=n_streams, mode=tz.ExecMode.Graph,
                         watchdog_s=args.watchdog_s, watchdog_k=args.watchdog_k,
                         graph_unroll=args.search_graph_unroll, pad_streams=max(pad, n_streams))


def _halo_verify(tz, rt, ctrl, halo):
    """verify(seq): one exchange of seq from a fresh grid of a new value generation, bad cells
    summed over ranks; verify(None): the grid as it stands (after the timed iterations)"""
    gen = [0]

    def verify(seq):
        if seq is not None:
            gen[0] = gen[0] % 3 + 1
            halo.init_grid(gen=gen[0])
            rt.device_sync()
            rt.prepare(seq)
            rt.run(1)
        rt.device_sync()
        return ctrl.allreduce_sum([float(halo.check_grid())])[0]
    return verify


def _reference_layout(tz, args, ctrl, device, branch):
    """The headline problem in the reference driver's storage: XYZQ (x fastest, one quantity per
    3-D block) with x = 0 at the start of the pitched row and the row pitch rounded up to 128 B
    (tenzing-mcts/examples/halo_run_strategy.hpp:42-49, 63-64: 528 doubles for 518 cells).
    Searched, verified and timed like the headline."""
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.utils.benchkit import search_record

    cfg = HaloConfig(n=args.n, neighbors=args.neighbors, fuse=args.fuse, order="xyzq",
                     transport=args.transport, ghost_align=-1)
    halo, graph = build_halo(cfg, ctrl, device)
    rt = _sub_runtime(tz, args, device, branch, args.streams)
    rec = search_record(tz, ctrl, rt, graph, args.streams, _halo_verify(tz, rt, ctrl, halo),
                        args.steps, args.warmup, seed=args.seed)
    if halo.uses_direct():
        rec["move_roof"] = halo.move_roof(20)
    rec["config"] = {"model": f"3D {'27' if args.neighbors == 26 else '7'}-point halo-exchange "
                              f"{args.n}^3 x {cfg.nq}q ghost {cfg.ghost}",
                     "storage_order": "xyzq", "x_origin": "row start (reference)",
                     "layout": halo.layout(), "streams": args.streams,
                     "halo_bytes_per_iter": halo.exchange_bytes()}
    del rt
    return rec


def spmv_via(names):
    """The x-halo transport of an SpMV schedule: "rccl" (the grouped exchange), "ipc" (kernel
    puts into the peers' receive buffers) or "local" (one rank: no halo)."""
    names = [n for n in names if not n.startswith("he_")]
    if any(n.endswith("exchange") for n in names):
        return "rccl"
    if any(n.endswith("put") for n in names):
        return "ipc"
    return "local"


def _baseline_configs(tz, args, ctrl, device, branch):
    """BASELINE.json configs 2 and 5 on this run's ranks, each searched briefly (MCTS, hipGraph
    candidates), verified and timed like the headline:
      spmv_c2:  CSR SpMV, m = 150,000, nnz = 10 m, band m / ranks, f32, 2 streams; between ranks
                the search chooses RCCL or IPC puts for the x halo
                (tenzing-dfs/examples/spmv.cu:86-117, tenzing-mcts/examples/spmv_run_strategy.cuh:44-125;
                BASELINE.md: 0.0094 ms on one rank, DFS over hipGraph candidates)
      fused_c5: that SpMV + the 26-neighbour 512^3 halo in one graph, 4 streams, the halo over
                the headline's transports (0.0544 ms on one rank)
    Each sub-record names the transports its winner used, the matrix's actual nnz (summed over
    ranks) and the RCCL communicator size."""
    from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused, build_spmv
    from tenzing_amd.utils.benchkit import remote_via, search_record

    recs = {}
    world = ctrl.size
    steps, warmup = max(args.steps, 20), max(args.warmup, 5)

    def spmv_verify(rt, s):
        def verify(seq):
            if seq is not None:
                s.reset_y()
                rt.device_sync()
                rt.prepare(seq)
                rt.run(1)
            rt.device_sync()
            err = ctrl.allreduce_max([s.check()])[0]
            return 0 if err < 1e-4 else 1
        return verify

    def spmv_facts(s, rec):
        names = [n for n in rec.get("schedule_gpu_ops", [])]
        via = spmv_via(names) if world > 1 else "local"
        return {"spmv_transport": via,
                "nnz": int(ctrl.allreduce_sum([float(s.local_nnz() + s.remote_nnz())])[0]),
                "nnz_target": s.args.nnz, "bw": s.args.bw, "ranks": world,
                "rccl_nranks": world if via == "rccl" else None,
                "spmv_transports_offered": ("rccl+ipc" if s.uses_rccl() and s.uses_ipc() else
                                            "rccl" if s.uses_rccl() else
                                            "ipc" if s.uses_ipc() else "local")}

    sc = SpmvConfig(m=150_000)
    s, g = build_spmv(sc, ctrl, device)
    rt = _sub_runtime(tz, args, device, branch, 2)
    rec = search_record(tz, ctrl, rt, g, 2, spmv_verify(rt, s), steps, warmup, mcts_iters=60,
                        search_unroll=8, seed=args.seed)
    rec["config"] = {"m": sc.m, "streams": 2, "dtype": "fp32",
                     "baseline_ms": 0.0094 if world == 1 else None, **spmv_facts(s, rec)}
    recs["spmv_c2"] = rec
    # config 2's workload stays alive until both sub-records are done: its RCCL communicators
    # are destroyed after the last RCCL operation of the run, never between two workloads'
    # (tests/gpu_rank_body.py: a teardown there hung or failed the next workload's first send)
    keep = (s, g)
    del rt

    grid = tuple(int(v) for v in args.rank_grid.lower().split("x")) if args.rank_grid else ()
    hc = HaloConfig(n=args.n, neighbors=26, order="qxyz", fuse="choice", transport=args.transport,
                    rank_grid=grid, relay=args.relay, hostsplit=args.hostsplit,
                    wide_puts=args.wide_puts, wide_put_blocks=args.wide_put_blocks,
                    copy_puts=args.copy_puts == "on")
    h, s, g = build_fused(hc, SpmvConfig(m=150_000), ctrl, device)
    rt = _sub_runtime(tz, args, device, branch, 4)
    # the largest tree of the BASELINE configs: greedy seeds measured before the search, one
    # with every group fused (the halo as one move on a stream of its own beside the SpMV)
    from tenzing_amd.search import choice_alternatives, greedy_schedule
    seeds = [greedy_schedule(g, tz.Platform(4), {"hs_launches": "hs_separate",
                                                 "*": ["allfused", "fused", "accum", "w16"]},
                             stream_for=lambda n: 1 if n.startswith("he_") else 0)]
    # one rank: the horizontally fused launch (move and SpMV in one kernel) as a second seed
    if "hs_onelaunch_i4" in choice_alternatives(g, "hs_launches"):
        seeds.append(greedy_schedule(g, tz.Platform(4), {"hs_launches": "hs_onelaunch_i4"}))
    hv, sv = _halo_verify(tz, rt, ctrl, h), spmv_verify(rt, s)

    def both(seq):
        if seq is not None:
            s.reset_y()
        b = hv(seq)
        return b + sv(None)
    rec = search_record(tz, ctrl, rt, g, 4, both, steps, warmup, mcts_iters=60, search_unroll=8,
                        seed=args.seed, seeds=seeds)
    names = rec.get("schedule_gpu_ops", [])
    rec["one_launch"] = next((n for n in names if n.startswith("hs_onelaunch")), None)
    rec["config"] = {"halo": f"{args.n}^3 x 3q ghost 3, 26 neighbours, qxyz", "spmv_m": 150_000,
                     "streams": 4, "baseline_ms": 0.0544 if world == 1 else None,
                     "rank_grid": list(h.rank_grid()),
                     "halo_transport": remote_via(names) or "direct",
                     "halo_rccl_nranks": h.rccl_nranks() or None,
                     **spmv_facts(s, rec)}
    recs["fused_c5"] = rec
    del rt, keep
    return recs


_STATE = {}  # what a failure report needs: the JSON line so far, the rank, the deadline


def _report_failure(why: str) -> None:
    """rank 0: print the JSON line as far as it got (marked partial, with the error), so that a
    run that fails still says how far it came; then disarm the deadline"""
    d = _STATE.get("deadline")
    if d is not None:
        d.cancel()
    out = _STATE.get("out")
    if _STATE.get("rank") == 0 and out is not None:
        out["partial"] = True
        out["error"] = why
        out["elapsed_s"] = round(time.time() - T_START, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    try:
        rc = main()
    except Exception as e:  # noqa: BLE001
        _report_failure(f"{type(e).__name__}: {e}")
        raise
    sys.exit(rc)
