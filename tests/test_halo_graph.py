"""Halo op-graph structure per transport and rank count (no GPU: graphs only, no setup).

Reference: src/halo_exchange/ops_halo_exchange.cu:33-84 (HaloExchange::add_to_graph builds
Pack -> Isend / Irecv -> Unpack chains per neighbour). Here self-neighbour directions become one
pack-free direct move each and remote directions keep pack -> RCCL shift -> unpack chains.
"""
import pytest


def _halo(tz, size, transport="auto", fuse="none", neighbors=26, rank=0):
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors, a.transport, a.fuse = neighbors, transport, fuse
    a.rank, a.size = rank, size
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
    names = _names(tz, g)
    assert sum(n.startswith("he_direct_") for n in names) == n_direct
    assert sum(n.startswith("he_pack_") for n in names) == 26 - n_direct
    assert sum(n.startswith("he_shift_") for n in names) == 26 - n_direct
    assert sum(n.startswith("he_unpack_") for n in names) == 26 - n_direct
    expect = {1: "direct", 8: "rccl"}.get(size, "direct+rccl")
    assert h.transport() == expect


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
