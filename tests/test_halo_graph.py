"""Halo op-graph structure per transport and rank count (no GPU: graphs only, no setup).

Reference: src/halo_exchange/ops_halo_exchange.cu:33-84 (HaloExchange::add_to_graph builds
Pack -> Isend / Irecv -> Unpack chains per neighbour). Here self-neighbour directions become one
pack-free direct move each and remote directions keep pack -> RCCL shift -> unpack chains.
"""
import pytest


def _halo(tz, size, transport="auto", fuse="none", neighbors=26, rank=0, hostsplit="off",
          ipc_grid=-1):
    # (host split off unless asked for: its alternatives would thin out the random rollouts
    # the older tests count transports in)
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.transport, a.fuse = neighbors, transport, fuse
    a.rank, a.size, a.hostsplit, a.ipc_grid = rank, size, hostsplit, ipc_grid
    h = tz.HaloExchange(a)
    g = tz.Graph()
    h.add_to_graph(g)
    return h, g


def _names(tz, g, seed=0):
    s = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
    return [o.name for o in s.ops() if isinstance(o, tz._tz.BoundGpuOp)]


@pytest.mark.parametrize("size,grid,n_direct", [(1, [1, 1, 1], 26), (2, [1, 1, 2], 8),
                                                (4, [1, 2, 2], 2), (8, [2, 2, 2], 0)])
def test_auto_transport_per_direction(tz, size, grid, n_direct):
    h, g = _halo(tz, size)
    assert list(h.rank_grid()) == grid
    direct = [i for i in range(h.ndirs()) if h.is_direct(i)]
    assert len(direct) == n_direct
    # locality is symmetric and means "self-neighbour"
    for i in range(h.ndirs()):
        assert h.is_direct(i) == h.is_direct(h.opposite(i)) == (h.neighbor(i) == 0)
    if size == 1:
        assert h.transport() == "direct"
    else:
        # remote directions: the search chooses between RCCL chains and IPC puts
        assert h.transport() == ("rccl+ipc" if n_direct == 0 else "direct+rccl+ipc")
        assert g.contains("he_remote")
    via = set()
    for seed in range(12):
        names = _names(tz, g, seed)
        assert sum(n.startswith("he_direct_") for n in names) == n_direct
        n_remote = 26 - n_direct
        if "he_wait_remote" in names:
            via.add("ipc")
            assert sum(n.startswith("he_put_") for n in names) == n_remote
            assert not any(n.startswith("he_shift_") for n in names)
        else:
            via.add("rccl" if n_remote else "none")
            for stage in ("he_pack_", "he_shift_", "he_unpack_"):
                assert sum(n.startswith(stage) for n in names) == n_remote
    assert via == ({"none"} if size == 1 else {"ipc", "rccl"})
    # forced RCCL: every direction (self-neighbours too) goes through RCCL
    hr, gr = _halo(tz, size, transport="rccl")
    assert hr.transport() == "rccl" and not any(hr.is_direct(i) for i in range(hr.ndirs()))


@pytest.mark.parametrize("fuse", ["all", "groups", "pack", "choice"])
@pytest.mark.parametrize("size", [1, 2, 8])
def test_fused_structures_roll_out(tz, fuse, size):
    h, g = _halo(tz, size, fuse=fuse)
    for seed in range(4):
        names = _names(tz, g, seed)
        assert len(names) == len(set(names))
        if h.uses_direct() and size > 1:
            # the self-neighbour moves are always fused into one op (except fuse=none)
            assert "he_direct_self" in names


def test_pipelined_ops_refuse_direct_directions(tz):
    h, _ = _halo(tz, 2)
    i = next(i for i in range(h.ndirs()) if h.is_direct(i))
    with pytest.raises(Exception, match="direct"):
        h.pack(i, 0)
    j = next(i for i in range(h.ndirs()) if not h.is_direct(i))
    with pytest.raises(Exception):
        h.direct(j, 0)


def test_copy_and_direct_need_self_neighbours(tz):
    for t in ("copy", "direct"):
        with pytest.raises(Exception, match="self-neighbours"):
            _halo(tz, 2, transport=t)
    h, _ = _halo(tz, 1, transport="copy")
    assert h.transport() == "copy" and not h.uses_direct()
    h, _ = _halo(tz, 2, transport="rccl")
    assert h.transport() == "rccl" and not h.uses_direct()


@pytest.mark.parametrize("mode", ["grid", "buffers"])
@pytest.mark.parametrize("fuse", ["none", "all", "choice"])
@pytest.mark.parametrize("size", [2, 8])
def test_ipc_transport_graph(tz, fuse, size, mode, monkeypatch):
    """ipc: self-neighbour moves, pack-free puts for remote directions, one arrival wait that
    every put precedes (and, in "buffers" mode, one unpack after the wait)"""
    h, g = _halo(tz, size, transport="ipc", fuse=fuse, ipc_grid=1 if mode == "grid" else 0)
    assert h.ipc_mode() == mode
    n_ipc = sum(h.is_ipc(i) for i in range(h.ndirs()))
    assert n_ipc == 26 - sum(h.is_direct(i) for i in range(h.ndirs()))
    assert h.transport() == ("ipc" if size == 8 else "direct+ipc")
    seen = set()
    for seed in range(12):
        names = _names(tz, g, seed)
        if any(n.startswith("he_rl") for n in names):
            # relay routing (2x2x2, buffers mode): checked in test_relay_routing_graph
            seen.add("relay")
            continue
        if any(n.startswith("he_hs") for n in names):
            # host split (buffers mode): checked in test_hostsplit_graph
            seen.add("hostsplit")
            continue
        if "he_wait_mx" in names:
            # buffers mode, mixed engines: + faces by kernel puts, - faces by copy-engine puts,
            # both before the one wait, one unpack after it
            seen.add("mx")
            w = names.index("he_wait_mx")
            assert names.index("he_put_mx") < w and names.index("he_copyput_mx") < w
            assert names.index("he_unpack_mx") > w
            assert not any(n.startswith(("he_pack_", "he_shift_")) for n in names)
            continue
        # buffers mode also offers copy-engine puts (pack locally, copy, signal) on the SDMA
        # engines ("cp_") or with the runtime's copy engine ("mc_"): ChoiceOp alternatives
        # whose op names differ
        v = ("cp_" if "he_wait_cp_remote" in names else
             "mc_" if "he_wait_mc_remote" in names else "")
        seen.add(v)
        w = names.index(f"he_wait_{v}remote")
        prefix = {"": "he_put_", "cp_": "he_copyput_", "mc_": "he_mcput_"}
        puts = [k for k, n in enumerate(names) if n.startswith(prefix[v])]
        assert puts and max(puts) < w
        assert not any(n.startswith(("he_pack_", "he_shift_")) for n in names)
        assert not any(n.startswith(p) for k, p in prefix.items() if k != v for n in names)
        unpacks = [k for k, n in enumerate(names) if n.startswith("he_unpack_")]
        if mode == "grid":
            assert not unpacks
        else:
            assert [names[k] for k in unpacks] == [f"he_unpack_{v}remote"] and unpacks[0] > w
        if fuse == "none":
            assert len(puts) == n_ipc
    seen.discard("relay")
    seen.discard("hostsplit")
    if mode == "grid":
        assert seen == {""}
    else:  # 12 rollouts: at least two of the four put transports
        assert len(seen) >= 2 and seen <= {"", "cp_", "mc_", "mx"}, seen


@pytest.mark.parametrize("transport", ["auto", "ipc"])
def test_relay_routing_graph(tz, transport, monkeypatch):
    """2x2x2 grid, ipc receive buffers: a share of every face can travel through the corner
    peer. Each relay alternative is putd / putc -> fwd -> wait -> unpack, the forward never
    ahead of the rank's own corner put; every rank builds the same names"""
    monkeypatch.setenv("TZ_IPC_GRID", "0")
    from tenzing_amd.models import HaloConfig

    graphs, hs = [], []
    for r in range(8):
        h = tz._tz.HaloExchange(HaloConfig(n=16, neighbors=26, order="qxyz", fuse="choice",
                                           transport=transport).args(r, 8, -1))
        g = tz.Graph()
        h.add_to_graph(g)
        hs.append(h)
        graphs.append(g)
    h, g = hs[0], graphs[0]
    assert h.uses_relay() and len(h.relay_faces()) == 6
    assert g.contains("he_remote")
    fracs, fwds = set(), set()
    for seed in range(60):
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
        names = [o.name for o in seq.ops() if isinstance(o, tz._tz.BoundGpuOp)]
        rl = [n for n in names if n.startswith("he_rl")]
        if not rl:
            continue
        t = rl[0][:len("he_rlNN")]
        fracs.add(t)
        fwd = f"{t}_fwd" if f"{t}_fwd" in names else f"{t}_fwdcp"
        k = {st: names.index(f"{t}_{st}") for st in ("putd", "putc", "wait", "unpack")}
        k["fwd"] = names.index(fwd)
        fwds.add(fwd[len(t) + 1:])
        assert k["putc"] < k["fwd"] < k["wait"] and k["putd"] < k["wait"] < k["unpack"]
        assert len(rl) == 5
        assert not any(n.startswith(("he_put_", "he_copyput_", "he_shift_")) for n in names)
        js = seq.json(True)
        for other in graphs[1:]:
            tz.OpIndex(other).sequence_from_json(js)
    assert fracs == {"he_rl15", "he_rl20", "he_rl25"} and fwds == {"fwd", "fwdcp"}
    # forced: the only remote transport
    a = HaloConfig(n=16, neighbors=6, order="qxyz", fuse="choice", transport="ipc", relay="force",
                   relay_fracs=(0.25,)).args(3, 8, -1)
    hf = tz._tz.HaloExchange(a)
    gf = tz.Graph()
    hf.add_to_graph(gf)
    assert hf.relay_faces() == list(range(6))
    for seed in range(5):
        names = [o.name for o in tz.random_rollout(tz.State(gf, tz.Platform(2)), seed).ops()
                 if isinstance(o, tz._tz.BoundGpuOp)]
        assert len(names) == 5 and ("he_rl25_fwd" in names or "he_rl25_fwdcp" in names)
        assert {f"he_rl25_{st}" for st in ("putd", "putc", "wait", "unpack")} <= set(names)


def test_relay_routing_needs_2x2x2_and_buffers(tz, monkeypatch):
    from tenzing_amd.models import HaloConfig

    monkeypatch.setenv("TZ_IPC_GRID", "0")
    for size in (2, 4):
        h = tz._tz.HaloExchange(HaloConfig(n=16, transport="ipc").args(0, size, -1))
        assert not h.uses_relay()
        with pytest.raises(Exception, match="relay"):
            tz._tz.HaloExchange(HaloConfig(n=16, transport="ipc", relay="force").args(0, size, -1))
    h = tz._tz.HaloExchange(HaloConfig(n=16, transport="ipc", relay="off").args(0, 8, -1))
    assert not h.uses_relay()
    monkeypatch.setenv("TZ_IPC_GRID", "1")
    assert not tz._tz.HaloExchange(HaloConfig(n=16, transport="ipc").args(0, 8, -1)).uses_relay()
    with pytest.raises(Exception, match="relay"):
        tz._tz.HaloExchange(HaloConfig(n=16, relay_fracs=(0.6,)).args(0, 8, -1))


@pytest.mark.parametrize("grid", [(1, 1, 8), (8, 1, 1), (2, 4, 1)])
def test_explicit_rank_grid_neighbours_are_symmetric(tz, grid):
    """an explicit rank grid (e.g. slabs) instead of the reference's prime-factor rule: every
    rank's neighbour in direction d sees this rank as its neighbour in direction -d"""
    from tenzing_amd.models import HaloConfig

    hs = [tz._tz.HaloExchange(HaloConfig(n=16, neighbors=26, rank_grid=grid).args(r, 8, -1))
          for r in range(8)]
    for r, h in enumerate(hs):
        assert list(h.rank_grid()) == list(grid)
        for i in range(h.ndirs()):
            q = h.neighbor(i)
            assert hs[q].neighbor(h.opposite(i)) == r


@pytest.mark.parametrize("size", [2, 4, 8])
@pytest.mark.parametrize("transport", ["auto", "rccl", "ipc"])
def test_every_rank_builds_the_same_op_names(tz, size, transport, monkeypatch):
    """schedules are broadcast from rank 0 by op name: every rank's graph must contain the same
    names for every alternative (per-peer groups included), in both IPC modes"""
    from tenzing_amd.models import HaloConfig

    for grid_mode in ("0", "1"):
        monkeypatch.setenv("TZ_IPC_GRID", grid_mode)
        graphs = []
        for r in range(size):
            h = tz._tz.HaloExchange(HaloConfig(n=32, neighbors=26, order="qxyz", fuse="choice",
                                               transport=transport).args(r, size, -1))
            g = tz.Graph()
            h.add_to_graph(g)
            graphs.append(g)
        for seed in range(25):
            js = tz.random_rollout(tz.State(graphs[0], tz.Platform(4)), seed).json(True)
            for g in graphs[1:]:
                tz.OpIndex(g).sequence_from_json(js)


def test_stencil_mode_graph(tz):
    """stencil mode: a ChoiceOp between "interior beside the exchange, shell after it" and
    "whole stencil after the exchange"; every rollout is race-free and keeps the stencil after
    the ghosts it reads"""
    from tenzing_amd.models import HaloConfig, build_halo

    h, g = build_halo(HaloConfig(n=32, neighbors=26, order="qxyz", fuse="choice", stencil=True),
                      setup=False)
    seen = set()
    for seed in range(40):
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
        names = [o.name for o in seq.ops()]
        st = [n for n in names if n.startswith("st_")]
        seen.add(tuple(sorted(st)))
        moves = [k for k, n in enumerate(names) if n.startswith("he_direct_")]
        if "st_full" in names:
            assert max(moves) < names.index("st_full")
        else:
            assert max(moves) < names.index("st_boundary")
    assert seen == {("st_full",), ("st_boundary", "st_interior")}


@pytest.mark.parametrize("size", [2, 8])
def test_hostsplit_graph(tz, size, monkeypatch):
    """buffers mode offers host split (a share of every face through node shared host memory,
    the rest as IPC puts), one alternative per share: both puts precede the one wait, the
    unpack follows it; forced, it is the only remote transport"""
    h, g = _halo(tz, size, fuse="choice", hostsplit="auto", ipc_grid=0)
    assert h.uses_hostsplit()
    from tenzing_amd.search import choice_alternatives, greedy_schedule
    alts = choice_alternatives(g, "he_remote")
    assert {"he_via_hs20", "he_via_hs30", "he_via_hs40"} <= set(alts)
    for alt in ("he_via_hs20", "he_via_hs30", "he_via_hs40"):
        for seed in range(3):
            st = tz.State(g, tz.Platform(3))
            seq = greedy_schedule(g, tz.Platform(3), {"he_remote": alt})
            names = [o.name for o in seq.ops()]
            p = alt[len("he_via_"):]
            d, hput, w, u = (names.index(f"he_{p}_{x}") for x in ("putd", "puth", "wait", "unpack"))
            assert max(d, hput) < w < u
            assert tz.verify(seq, tz.resolve_graph(g, seq), 3) == []
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.fuse, a.rank, a.size, a.hostsplit = 26, "choice", 0, size, "force"
    a.ipc_grid = 0
    hf = tz.HaloExchange(a)
    gf = tz.Graph()
    hf.add_to_graph(gf)
    assert choice_alternatives(gf, "he_remote") == ["he_via_hs10", "he_via_hs20", "he_via_hs30", "he_via_hs40"]
    # grid mode has no receive buffers: not offered
    hg, _ = _halo(tz, size, hostsplit="auto", ipc_grid=1)
    assert not hg.uses_hostsplit()


@pytest.mark.parametrize("parts", [1, 3, 4, 8])
def test_host_share_chunks_tile_the_box(tz, parts):
    """the host share travels in chunks: in order along the box's largest dimension, covering
    every row of it exactly once, each chunk's buffer on a 128-B boundary behind the previous
    one; sender and receiver cut boxes of one shape the same way"""
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.rank, a.size = 26, 0, 2
    h = tz.HaloExchange(a)
    for i in range(h.ndirs()):
        b = h.pack_box(i)
        b["buf"] = 1 << 20  # a fake base address: only the offsets matter
        cs = tz.HaloExchange.chunk_box(b, parts)
        n = [b["n1"], b["n2"], b["n3"]]
        k = max((2, 1, 0), key=lambda j: n[j])  # the largest, slower on ties
        assert len(cs) == min(parts, n[k])
        rows = [c[("n1", "n2", "n3")[k]] for c in cs]
        assert sum(rows) == n[k] and max(rows) - min(rows) <= 1
        stride = b[("s1", "s2", "s3")[k]]
        at, off = 0, b["buf"]
        for c in cs:
            assert c["grid_off"] == b["grid_off"] + at * stride
            assert c["buf"] == off and (c["buf"] - b["buf"]) % 128 == 0
            for j in range(3):
                if j != k:
                    assert c[("n1", "n2", "n3")[j]] == n[j]
            at += c[("n1", "n2", "n3")[k]]
            elems = c["len"] * c["n1"] * c["n2"] * c["n3"]
            off += ((elems + 15) // 16 * 16) * 8
        u = h.unpack_box(h.opposite(i))
        u["buf"] = 0
        assert [(c["n1"], c["n2"], c["n3"]) for c in tz.HaloExchange.chunk_box(u, parts)] == \
            [(c["n1"], c["n2"], c["n3"]) for c in cs]


def test_hostsplit_chunks_option(tz):
    a = tz.HaloArgs()
    assert a.hostsplit_chunks == 1
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.rank, a.size, a.hostsplit_chunks = 26, 0, 2, 0
    with pytest.raises(Exception, match="hostsplit_chunks"):
        tz.HaloExchange(a)


def test_host_share_chunk_count_is_the_same_for_every_face(tz):
    """at 24^3 cells a 10 % share of a y or z face has only 3 rows to cut along, an x face 24:
    every face then travels in 3 chunks (not 4 for x), so a chunk launch holds all faces and the
    positional arrival counters stay aligned when the schedule switches to a 20 % share (4)"""
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 24
    a.neighbors, a.order, a.rank, a.size, a.hostsplit_chunks = 26, "qxyz", 0, 8, 4
    h = tz.HaloExchange(a)
    assert h.hostsplit_parts(0.1) == 3 and h.hostsplit_parts(0.2) == 4
    a.hostsplit_chunks = 1
    assert tz.HaloExchange(a).hostsplit_parts(0.2) == 1


@pytest.mark.parametrize("fuse", ["none", "all", "groups", "choice"])
@pytest.mark.parametrize("grid_mode", ["1", "0"])
def test_wide_puts_are_a_transport_alternative(tz, monkeypatch, fuse, grid_mode):
    """wide_puts="on": the IPC put again with more workgroups per box, as its own he_remote
    alternative ("he_via_ipcw"); its ops carry "he_putw_" / "w_" and never mix with the
    default put's. Graph-only builds offer it only when asked ("auto" decides at setup)."""
    from tenzing_amd.search import choice_alternatives, greedy_schedule

    a = tz.HaloArgs()
    a.ipc_grid = int(grid_mode)
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.fuse, a.rank, a.size, a.hostsplit, a.relay = 26, fuse, 0, 8, "off", "off"
    h0 = tz.HaloExchange(a)
    g0 = tz.Graph()
    h0.add_to_graph(g0)
    assert not h0.uses_wide_puts()
    assert "he_via_ipcw" not in choice_alternatives(g0, "he_remote")
    a.wide_puts = "on"
    h = tz.HaloExchange(a)
    g = tz.Graph()
    h.add_to_graph(g)
    assert h.uses_wide_puts()
    assert "he_via_ipcw" in choice_alternatives(g, "he_remote")
    p = tz.Platform(3)
    s = greedy_schedule(g, p, {"he_remote": "he_via_ipcw"})
    names = [o.name for o in s.ops() if isinstance(o, tz._tz.BoundGpuOp)]
    wide = [n for n in names if n.startswith("he_putw_")]
    assert wide and not any(n.startswith("he_put_") for n in names)
    w = names.index("he_wait_w_remote")
    assert max(names.index(n) for n in wide) < w
    if fuse == "none":
        assert len(wide) == 26
    assert tz.verify(s, tz.resolve_graph(g, s), 3) == []
    kinds = {o.kind for o in s.ops()}
    assert kinds & {"HaloWidePut", "HaloWidePutGroup"}


def test_wide_put_args_are_checked(tz):
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.wide_puts = "sometimes"
    with pytest.raises(Exception, match="wide_puts"):
        tz.HaloExchange(a)
    a.wide_puts, a.wide_put_blocks = "on", 0
    with pytest.raises(Exception, match="wide_put_blocks"):
        tz.HaloExchange(a)
    a.wide_put_blocks = 128
    assert '"wide_put_blocks":128' in a.json().replace(" ", "")


def test_wide_put_offer_on_a_fake_topology(tz):
    """the per-rank decision behind wide_puts="auto": peers on other GPUs (another PCI bus id, or
    peer memory the runtime maps on another device) offer the wide put; loopback ranks (every
    peer on my bus / device) do not; unknown facts decide nothing"""
    offered = tz._tz.HaloExchange.wide_puts_offered
    me = "0000:05:00.0"
    # an 8-GPU node: the IPC peers sit on other buses, whatever the mapping reports
    assert offered("auto", me, ["0000:15:00.0", "0000:65:00.0"], 0, [0, 0])
    # ... or only the mapping knows (bus ids unavailable)
    assert offered("auto", "", ["", ""], 0, [3])
    # loopback: all on my GPU
    assert not offered("auto", me, [me, me.upper().lower()], 0, [0, 0])
    assert not offered("auto", me, ["", me], 0, [-1])
    # forced either way
    assert offered("on", me, [me], 0, [0])
    assert not offered("off", me, ["0000:15:00.0"], 0, [1])


def test_link_matrix_needs_pairs_and_whole_rows(tz):
    """the all-pairs link probe: one rank has no pairs (nothing touches a GPU); transfer sizes
    must be whole 32 KiB rows"""
    lm = tz._tz.link_matrix(tz._tz.SelfCtrl(), 1 << 20, 2)
    assert lm["why"] == "one rank: no pairs" and lm["put_GBps"] == [[-1.0]]
    with pytest.raises(Exception, match="multiple of 32768"):
        tz._tz.link_matrix(tz._tz.SelfCtrl(), 1000, 2)


@pytest.mark.parametrize("order,align", [("qxyz", -2), ("xyzq", 16), ("xyzq", -1)])
def test_unpack_widening_covers_only_row_padding(tz, order, align):
    """the unpack's x-ghost rows may be widened to whole ghost_align units, over row padding
    only: never into the interior, never past the row; none without line-aligned ghosts"""
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 64
    a.ghost, a.nq, a.neighbors, a.order, a.ghost_align = 3, 3, 26, order, align
    h = tz.HaloExchange(a)
    lay = h.layout()
    pitch, q, g, xoff = lay["row_pitch_elems"], a.nq, a.ghost, lay["x_offset_cells"]
    # elements of a row: padding [0, lo), ghost-low, interior, ghost-high, padding [hi, pitch)
    if order == "qxyz":
        lo, hi = q * xoff, q * (xoff + a.nx + 2 * g)
    else:
        lo, hi = xoff, xoff + a.nx + 2 * g
    widened = 0
    for i in range(h.ndirs()):
        b = h.unpack_box(i)
        dx = h.dir(i)[0]
        x0 = b["grid_off"] % pitch
        if dx == 0 or align == -1:
            assert b["lead"] == b["trail"] == 0, (i, b)
            continue
        assert b["lead"] <= x0 - 0 and x0 - b["lead"] >= 0
        if b["lead"]:
            assert dx < 0 and x0 - b["lead"] >= 0 and x0 <= lo + (q * g if order == "qxyz" else g)
        if b["trail"]:
            assert dx > 0 and x0 + b["len"] + b["trail"] <= pitch and x0 + b["len"] >= hi
        # whole units, 16-B aligned
        assert (x0 - b["lead"]) % 2 == 0 and (b["lead"] + b["len"] + b["trail"]) % 2 == 0
        widened += b["lead"] + b["trail"] > 0
    assert (widened > 0) == (align != -1)
