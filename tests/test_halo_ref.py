"""The independent torch model of a completed exchange (tenzing_amd/utils/halo_ref.py), checked
on the CPU against a cell-by-cell loop, and the storage strides the workload reports."""
import itertools

import pytest
import torch

from tenzing_amd.utils import halo_ref


def _naive(field, coords, n, g, neighbors, before):
    nq = field.shape[0]
    ext = field.shape[1:]
    out = before.clone()
    for z, y, x in itertools.product(*(range(k + 2 * g) for k in n)):
        ghosts = sum(int(i < g or i >= k + g) for i, k in zip((z, y, x), n))
        if neighbors == 6 and ghosts >= 2:
            continue
        gz, gy, gx = ((c * k + i - g) % e for c, k, i, e in zip(coords, n, (z, y, x), ext))
        for q in range(nq):
            out[q, z, y, x] = field[q, gz, gy, gx]
    return out


@pytest.mark.parametrize("neighbors", [6, 26])
@pytest.mark.parametrize("coords", [(0, 0, 0), (1, 0, 1)])
def test_expected_block_matches_a_cell_loop(neighbors, coords):
    n, g, grid = (3, 4, 5), 2, (2, 1, 2)
    field = halo_ref.global_field(2, tuple(p * k for p, k in zip(grid, n)), seed=5)
    before = torch.full((2, *(k + 2 * g for k in n)), -2.5, dtype=torch.float64)
    got = halo_ref.expected_block(field, coords, n, g, neighbors, before)
    assert torch.equal(got, _naive(field, coords, n, g, neighbors, before))


def test_field_is_the_same_for_one_seed():
    a = halo_ref.global_field(3, (4, 4, 4), seed=1)
    assert torch.equal(a, halo_ref.global_field(3, (4, 4, 4), seed=1))
    assert not torch.equal(a, halo_ref.global_field(3, (4, 4, 4), seed=2))


@pytest.mark.parametrize("pitch_pad", [0, 16])
@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
@pytest.mark.parametrize("ghost_align", [-1, 0, 8, 16])
def test_reported_strides_address_the_grid(tz, order, ghost_align, pitch_pad):
    """every logical cell has its own storage element inside the grid, and x runs along the
    fastest axis of its layout (checked without a GPU: the workload is not set up)"""
    from tenzing_amd.models import HaloConfig, build_halo

    cfg = HaloConfig(n=6, neighbors=26, order=order, ghost_align=ghost_align, transport="direct",
                     pitch_pad=pitch_pad)
    h, _ = build_halo(cfg, tz.SelfCtrl(), setup=False)
    lay = h.layout()
    st, shape = lay["strides_qzyx"], lay["shape_qzyx"]
    assert tuple(shape) == (3, 12, 12, 12) and lay["ghost"] == 3
    storage = torch.zeros(h.grid_elems(), dtype=torch.int32)
    view = halo_ref.logical_view(storage, lay)
    view += 1  # every logical cell once
    assert int(storage.sum()) == 3 * 12 ** 3 and int(storage.max()) == 1
    assert st[3] == (1 if order == "xyzq" else 3)
    assert lay["row_pitch_elems"] == st[2] and st[2] % 16 == 0
    if ghost_align == -1:
        assert lay["x_offset_cells"] == 0
    if ghost_align in (8, 16) and order == "xyzq":
        # the first interior cell (x = ghost) starts an aligned run
        assert (lay["x_offset_cells"] + 3) % ghost_align == 0


@pytest.mark.parametrize("coords", [(0, 0, 0), (1, 0, 1), (1, 1, 1)])
def test_hashed_block_is_the_padded_global_field(coords):
    """the per-rank hashed block equals circular padding of the materialized hashed field"""
    n, g, grid, nq = (3, 4, 5), 2, (2, 2, 2), 2
    ext = tuple(p * k for p, k in zip(grid, n))
    iz, iy, ix = (torch.arange(e).view(s) for e, s in zip(ext, ((-1, 1, 1), (1, -1, 1), (1, 1, -1))))
    field = torch.stack([halo_ref.hashed_values(q, iz, iy, ix, ext, 7) for q in range(nq)])
    assert 0 <= float(field.min()) and float(field.max()) < 1
    assert field.unique().numel() == field.numel()
    before = torch.full((nq, *(k + 2 * g for k in n)), -2.5, dtype=torch.float64)
    want = halo_ref.expected_block(field, coords, n, g, 26, before)
    assert torch.equal(halo_ref.hashed_block(nq, coords, n, ext, g, 7), want)
    assert not torch.equal(halo_ref.hashed_block(nq, coords, n, ext, g, 8), want)
