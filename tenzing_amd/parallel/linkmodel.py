"""Link-aware cost model of the multi-GPU halo exchange, for hardware-free searches.

The discrete-event simulator (``SimBenchmarker`` with ``SimParams.link_model``) times a GPU op
that reports its traffic (``GpuOp.traffic()``: bytes per shared resource and engine) as its
fixed latency plus, over its resources, the longest ``bytes / rate``, where ``rate`` is the
engine's own rate capped by the resource's capacity shared with the transfers already active
on it. The halo ops report per-peer xGMI bytes (kernel puts, wide puts, copy engines, RCCL,
relay hops through the corner peer), PCIe bytes (host split) and local HBM bytes.

``link_sim_params`` fills the rates from what a multi-GPU bench run measured (its
``link_probe`` and ``link_matrix`` fields), so that a search over recorded link rates runs on a
CPU. ``headline_graph`` builds the bench's N-rank tree for one rank without a GPU, and
``transport_seeds`` the bench's one-schedule-per-transport seeds.

Reference: tenzing-mcts replays recorded timings without hardware (CsvBenchmarker,
src/benchmarker.cpp:169-223); the MCTS loop is tenzing-mcts/include/tenzing/mcts/mcts.hpp:154-326.
"""
from __future__ import annotations

from .. import _tz

# xGMI: 7 links of ~153 GB/s peak per direction per MI355X; what one transfer reaches depends on
# the engine (CU stores at the default / wide workgroup count, SDMA, RCCL)
DEFAULT_ENGINE_GBPS = {"kernel": 5000.0, "put": 60.0, "wide": 90.0, "sdma": 50.0, "memcpy": 50.0,
                       "rccl": 50.0, "host": 40.0}
DEFAULT_RESOURCE_GBPS = {"hbm": 5000.0, "xgmi": 120.0, "pcie": 50.0}


def link_sim_params(probe: dict | None = None, matrix: dict | None = None, noise: float = 0.0,
                    seed: int = 0, graph: bool = True, **engine_overrides) -> "_tz.SimParams":
    """SimParams with the link-aware model on. ``probe``: a bench record's ``link_probe`` (one
    transfer's GB/s per transport over one link, and both faces of an axis at once, which
    bounds the link's capacity); ``matrix``: its ``link_matrix`` (every ordered pair, all ranks
    sending at once: per-link capacities ``xgmi:<peer>`` of rank 0's links). Missing fields keep
    the defaults; ``engine_overrides`` (e.g. ``put=70``) win over both. ``graph``: time the
    sequence as a back-to-back hipGraph replay (``SimParams.graph``: device-side kernel gaps and
    fork/join costs measured on MI355X), the way the bench searches and times; False: as eager
    launches from the host."""
    p = _tz.SimParams()
    p.link_model = True
    p.graph = graph
    p.noise = noise
    p.seed = seed
    eng = dict(DEFAULT_ENGINE_GBPS)
    res = dict(DEFAULT_RESOURCE_GBPS)
    if probe:
        rates = probe.get("GBps") or {}
        for key, name in (("put", "put"), ("put_wide", "wide"), ("sdma", "sdma"),
                          ("memcpy", "memcpy"), ("rccl", "rccl")):
            if rates.get(key):
                eng[name] = float(rates[key])
        pair = [v for v in (probe.get("pair_GBps") or {}).values() if v]
        if pair:  # both faces of one axis at once over the same link: at least this much
            res["xgmi"] = max(res["xgmi"], float(max(pair)))
    if matrix and matrix.get("put_GBps") and not matrix.get("why"):
        row = matrix["put_GBps"][0]
        for q, v in enumerate(row):
            if v and v > 0:
                res[f"xgmi:{q}"] = max(float(v), eng["put"])
    eng.update({k: float(v) for k, v in engine_overrides.items()})
    p.engine_GBps = eng
    p.resource_GBps = res
    return p


def relay_share(face_GBps: float = 1.0, corner_GBps: float = 1.0) -> float:
    """The relayed share f* of every face that balances the 2x2x2 grid's busiest links.

    Without relaying, each face link carries both faces of its axis (2 B per exchange, B = one
    face). Relaying a share f of all 6 faces through the corner peer puts 6 f B on the corner link
    and leaves (1 - f) 2 B on each face link, so the busiest link takes
    max((1 - f) 2 B / r_face, 6 f B / r_corner), smallest at f* = r_corner / (r_corner + 3 r_face):
    0.25 at equal link rates, i.e. 0.75 of a face pair on every busy link. (The second hop runs
    over a yz-style diagonal link, which otherwise carries only edges: 2 f B, never the busiest.)"""
    if face_GBps <= 0 or corner_GBps <= 0:
        raise ValueError("link rates must be positive")
    return corner_GBps / (corner_GBps + 3.0 * face_GBps)


def relay_fracs_offered(f_star: float, base=(0.15, 0.2)) -> tuple:
    """The relay shares the search chooses among: the fixed ones (0.2 balances the links when the
    forward waits for the whole share to arrive, docs/RESULTS.md) and the link model's f*,
    clamped into the range the relay accepts, (0, 0.5)."""
    f = min(0.45, max(0.05, round(float(f_star), 3)))
    return tuple(sorted(set(base) | {f}))


def relay_share_from_record(record: dict):
    """f* from a multi-GPU bench record's own link matrix (rank 0's put rates to its face peers
    and to its corner peer, every pair sending at once), or None when the record has no 2x2x2
    grid or no matrix."""
    cfg = record.get("config") or {}
    if list(cfg.get("rank_grid") or []) != [2, 2, 2]:
        return None
    m = (record.get("link_matrix") or {}).get("put_GBps")
    if not m or (record.get("link_matrix") or {}).get("why"):
        return None
    row = m[0]
    # rank r = x + 2 y + 4 z in the 2x2x2 grid (HaloExchange's rank order): rank 0's face peers
    # are 1, 2 and 4, its corner peer 7
    face = [row[q] for q in (1, 2, 4) if row[q] and row[q] > 0]
    corner = row[7] if row[7] and row[7] > 0 else None
    if not face or corner is None:
        return None
    return relay_share(sum(face) / len(face), corner)


def graph_params_from_probe(params, branch: dict | None):
    """``params`` with its hipGraph join cost taken from a bench record's ``graph_branch_probe``
    (the padding in use): the unrolled 3-branch replay's time over the one-branch replay's is
    one join of 3 streams, i.e. graph_join_us + graph_wait_us (SimParams.graph). Unchanged
    without an unrolled probe."""
    if not branch:
        return params
    probe = None
    for t in branch.get("tried") or []:
        if t.get("pad_streams") == branch.get("pad_streams") and t.get("probe"):
            probe = t["probe"]
    u = (probe or {}).get("unrolled") or {}
    if not u.get("all_us") or not u.get("one_us") or (probe or {}).get("branches") != 3:
        return params
    join3 = float(u["all_us"]) - float(u["one_us"])
    if join3 > 0:
        params.graph_join_us = max(1.0, join3 - params.graph_wait_us)
    return params


def headline_graph(rank: int, size: int, n: int = 512, neighbors: int = 26, order: str = "qxyz",
                   wide_puts: str = "on", relay: str = "auto", hostsplit: str = "auto",
                   ipc_grid=None):
    """(halo, graph) of one rank of the bench's N-rank tree, built without a GPU: every remote
    transport offered (RCCL, kernel / wide / copy-engine puts, their mix, relays, host split)
    as the top-level ChoiceOp, per-direction or fused groups below it. ipc_grid=0 (or
    TZ_IPC_GRID=0) for the receive-buffer transports (copy engines, relay, host split)."""
    from ..models import HaloConfig

    cfg = HaloConfig(n=n, neighbors=neighbors, order=order, fuse="choice", transport="auto",
                     wide_puts=wide_puts, relay=relay, hostsplit=hostsplit, ipc_grid=ipc_grid)
    h = _tz.HaloExchange(cfg.args(rank, size, -1))
    g = _tz.Graph()
    h.add_to_graph(g)
    return h, g


def transport_seeds(graph, platform, streams: int):
    """The bench's seeds (bench.py, --seed-transports): one greedy schedule per remote transport
    of the ``he_remote`` choice, every group fused, direct (self) moves on stream 1."""
    from ..search import choice_alternatives, greedy_schedule

    seeds, alts = [], []
    for alt in choice_alternatives(graph, "he_remote"):
        try:
            seeds.append(greedy_schedule(
                graph, platform, {"he_remote": alt, "*": ["allfused", "fused"]},
                stream_for=lambda n: 1 if n.startswith("he_direct") and streams > 1 else 0))
            alts.append(alt)
        except RuntimeError:
            continue
    return seeds, alts


def tree_stats(graph, platform, rollouts: int = 50, seed: int = 0) -> dict:
    """Size of the decision tree: decisions per complete schedule and the mean / max number of
    alternatives at each step, over random rollouts."""
    import random

    rng = random.Random(seed)
    depths, widths = [], []
    for _ in range(rollouts):
        st = _tz.State(graph, platform)
        d = 0
        while not st.complete():
            ds = st.get_decisions()
            widths.append(len(ds))
            st = st.apply(ds[rng.randrange(len(ds))])
            d += 1
        depths.append(d)
    log10 = sum(__import__("math").log10(w) for w in widths) / max(1, len(depths))
    return {"rollouts": rollouts, "depth_mean": sum(depths) / len(depths), "depth_max": max(depths),
            "branching_mean": sum(widths) / len(widths), "branching_max": max(widths),
            "log10_paths_per_rollout": round(log10, 1)}


def sim_seeds(graph, platform, k: int = 2, iters: int = 400, params=None, exclude=(), seed: int = 0):
    """The ``k`` best distinct schedules of a hardware-free MCTS (FastMin, ``iters`` iterations)
    under the link-aware model: seeds for a measured search, so that it starts from structures
    the model ranks well (stream splits, transport mixes) besides the greedy per-transport ones.
    ``exclude``: sequences already seeded (skipped by canonical key). Returns
    [(sequence, model_us)], best first. One process, no GPU, no collectives."""
    if k <= 0:
        return []
    p = params if params is not None else link_sim_params()
    o = _tz.MctsOpts()
    o.n_iters = iters
    o.strategy = "FastMin"
    o.seed = seed
    o.bench = _tz.BenchOpts(n_iters=2, max_retries=1, target_secs=0.001)
    if exclude:
        o.seed_schedules = list(exclude)
    res = _tz.mcts_explore(graph, platform, _tz.SimBenchmarker(platform.n_streams, p), _tz.SelfCtrl(), o)
    skip = {s.canonical_key() for s in exclude}
    out, keys = [], set(skip)
    for i in sorted(range(len(res.sims)), key=lambda i: res.sims[i].res.pct10):
        sq = res.sims[i].seq
        key = sq.canonical_key()
        if key in keys:
            continue
        keys.add(key)
        out.append((sq, res.sims[i].res.pct10 * 1e6))
        if len(out) >= k:
            break
    return out


def find_record(doc):
    """The first bench record (a dict with ``link_probe``) in ``doc``: a record, a list of them,
    or any JSON nesting them (a driver's scaling file); None if there is none."""
    if isinstance(doc, dict):
        if "link_probe" in doc:
            return doc
        doc = list(doc.values())
    if isinstance(doc, list):
        for v in doc:
            r = find_record(v)
            if r is not None:
                return r
    return None


def load_records(path: str) -> list:
    """Every bench record with a ``link_probe`` in a file: one JSON document or JSON lines."""
    import json

    text = open(path).read()
    try:
        docs = [json.loads(text)]
    except ValueError:
        docs = [json.loads(x) for x in text.splitlines() if x.strip().startswith("{")]
    out = []

    def walk(o):
        if isinstance(o, dict):
            if "link_probe" in o:
                out.append(o)
                return
            o = list(o.values())
        if isinstance(o, list):
            for v in o:
                walk(v)
    walk(docs)
    return out


def model_report(record: dict, params=None) -> dict:
    """How well the link-aware replay model, calibrated on a multi-GPU bench record's own
    ``link_probe`` / ``link_matrix`` (and its join cost on ``graph_branch_probe``), predicts that record's measured seeds: for every remote
    transport the bench seeded (one greedy schedule each, ``seeded_pct10_ms``), the model's time
    of the same schedule on rank 0's graph beside the measured one, and the rank correlation of
    the two orders. Needs no GPU."""
    from ..utils.benchkit import remote_via

    cfg = record.get("config") or {}
    size = int(record.get("n_gpus") or 1)
    streams = int(cfg.get("streams") or 4)
    p = params if params is not None else graph_params_from_probe(
        link_sim_params(record.get("link_probe"), record.get("link_matrix")),
        record.get("graph_branch_probe"))
    # the record's IPC mode (puts into the peer's grid, or into receive buffers: the copy-engine,
    # relay and host-split transports)
    h, g = headline_graph(0, size, n=int(cfg.get("seq_len") or 512),
                          neighbors=int(cfg.get("neighbors") or 26),
                          order=cfg.get("storage_order") or "qxyz",
                          wide_puts="on" if record.get("wide_puts_offered", True) else "off",
                          relay="auto" if record.get("relay_offered", True) else "off",
                          hostsplit="auto" if record.get("hostsplit_offered", True) else "off",
                          ipc_grid=1 if record.get("ipc_mode") == "grid" else 0)
    platform = _tz.Platform(streams)
    seeds, _ = transport_seeds(g, platform, streams)
    measured = record.get("seeded_pct10_ms") or {}
    rows = []
    for sq in seeds:
        via = remote_via([o.name for o in sq.ops()]) or "none"
        model_us = _tz.SimExecutor(streams, p).run_once(sq)
        rows.append({"transport": via, "model_us": round(model_us, 1),
                     "measured_us": round(measured[via] * 1e3, 1) if via in measured else None})
    both = [r for r in rows if r["measured_us"] is not None]
    for r in both:
        r["measured_over_model"] = round(r["measured_us"] / r["model_us"], 3)

    def ranks(v):
        order = sorted(range(len(v)), key=lambda i: v[i])
        out = [0.0] * len(v)
        for k, i in enumerate(order):
            out[i] = float(k)
        return out

    rho = None
    if len(both) >= 3:
        a, b = ranks([r["model_us"] for r in both]), ranks([r["measured_us"] for r in both])
        n = len(both)
        rho = 1 - 6 * sum((x - y) ** 2 for x, y in zip(a, b)) / (n * (n * n - 1))
    best_model = min(rows, key=lambda r: r["model_us"])["transport"] if rows else None
    best_meas = min(both, key=lambda r: r["measured_us"])["transport"] if both else None
    return {"n_gpus": size, "streams": streams, "engine_GBps": dict(p.engine_GBps),
            "resource_GBps": dict(p.resource_GBps), "seeds": rows, "spearman": rho,
            "best_by_model": best_model, "best_measured": best_meas,
            "record_value_ms": record.get("value"),
            "record_transport": record.get("schedule_transport"),
            "model_seeded": record.get("model_seeded")}


def _main(argv=None) -> int:
    import argparse
    import json

    ap = argparse.ArgumentParser(
        prog="python -m tenzing_amd.parallel.linkmodel",
        description="model vs measured for every multi-GPU bench record in a file")
    ap.add_argument("record", help="bench JSON lines, one record, or a file nesting records")
    a = ap.parse_args(argv)
    recs = [r for r in load_records(a.record) if (r.get("n_gpus") or 1) > 1]
    if not recs:
        print(f"no multi-GPU bench record with a link_probe in {a.record}")
        return 1
    for r in recs:
        print(json.dumps(model_report(r)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
