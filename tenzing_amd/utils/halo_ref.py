"""An independent model of a completed halo exchange, in plain torch.

`HaloExchange.check_grid` counts wrong cells with a device kernel whose expected values come
from the same geometry code as the exchange itself (`csrc/kernels/halo_kernels.hip`,
`halo_expect`). The reference has no halo output or fixture to compare against (its halo driver
does not build at HEAD: `include/tenzing/graph.hpp:62-65` vs
`src/halo_exchange/ops_halo_exchange.cu:50`), so this module pins the exchange to a model that
shares nothing with the native code:

- the global field is random (not an encoded coordinate): drawn by a torch generator from a
  seed, the same on every rank, or (any size) a multiplicative hash of each cell's global index
  that each rank evaluates for its own block only;
- the expected local block is a slice of the field padded periodically by ``torch.nn.functional
  .pad(mode="circular")``;
- the grid is read back through the storage strides the workload reports
  (``HaloExchange.layout()``), so the layout itself is checked as well.

The semantics are those of the reference's exchange (`src/halo_exchange/ops_halo_exchange.cu`):
periodic boundaries over the rank grid, ghost width ``g`` on every side, 6 neighbours fill the
face ghosts only, 26 fill faces, edges and corners.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def global_field(nq: int, extent_zyx, seed: int) -> torch.Tensor:
    """random fp64 field (nq, GZ, GY, GX), identical on every rank for one seed"""
    gen = torch.Generator().manual_seed(int(seed))
    return torch.rand((nq, *extent_zyx), generator=gen, dtype=torch.float64)


_P = 2147483647  # 2^31 - 1
_A = 48271


def hashed_values(q: int, gz, gy, gx, extent_zyx, seed: int) -> torch.Tensor:
    """a pseudo-random value in [0, 1) for every global cell (q, gz, gy, gx) (broadcastable int64
    tensors of wrapped coordinates): two multiplicative rounds modulo 2^31 - 1 of the cell's
    linear index. Any rank computes any cell's value without the global field, so the model
    scales to any rank count; cells closer than 2^31 - 1 in the linear index never share a value"""
    GZ, GY, GX = (int(e) for e in extent_zyx)
    idx = ((q * GZ + gz) * GY + gy) * GX + gx
    h = ((idx % _P) * _A + (int(seed) % 65536) * 16807 + 12345) % _P
    h = (h * _A) % _P
    return h.to(torch.float64) / _P


def hashed_block(nq: int, coords_zyx, n_zyx, extent_zyx, g: int, seed: int,
                 device="cpu") -> torch.Tensor:
    """the padded block (nq, nz+2g, ny+2g, nx+2g) of the rank at `coords_zyx` in the periodic
    hashed field: its interior is what the rank holds, all of it what a 26-neighbour exchange
    leaves"""
    ax = []
    for k, (c, n, e) in enumerate(zip(coords_zyx, n_zyx, extent_zyx)):
        i = (torch.arange(n + 2 * g, device=device, dtype=torch.int64) + (c * n - g)) % int(e)
        shape = [1, 1, 1]
        shape[k] = n + 2 * g
        ax.append(i.view(shape))
    out = torch.empty((nq, *(n + 2 * g for n in n_zyx)), dtype=torch.float64, device=device)
    for q in range(nq):
        out[q] = hashed_values(q, ax[0], ax[1], ax[2], extent_zyx, seed)
    return out


def ghost_class(n_zyx, g: int) -> torch.Tensor:
    """number of ghost axes (0 interior, 1 face, 2 edge, 3 corner) of every padded cell (z, y, x)"""
    out = None
    for axis, n in enumerate(n_zyx):
        i = torch.arange(n + 2 * g)
        ghost = ((i < g) | (i >= n + g)).to(torch.int8)
        shape = [1, 1, 1]
        shape[axis] = n + 2 * g
        ghost = ghost.view(shape)
        out = ghost if out is None else out + ghost
    return out


def expected_block(field: torch.Tensor, coords_zyx, n_zyx, g: int, neighbors: int,
                   before: torch.Tensor) -> torch.Tensor:
    """the padded local block (nq, nz+2g, ny+2g, nx+2g) of the rank at `coords_zyx` after a
    complete exchange; cells the exchange does not fill keep their `before` values"""
    padded = F.pad(field.unsqueeze(0), (g, g, g, g, g, g), mode="circular")[0]
    sl = [slice(None)]
    for c, n in zip(coords_zyx, n_zyx):
        sl.append(slice(c * n, c * n + n + 2 * g))
    block = padded[tuple(sl)].clone()
    if neighbors == 6:
        keep = (ghost_class(n_zyx, g) >= 2).to(block.device).expand_as(block)
        block[keep] = before[keep]
    return block


def logical_view(storage: torch.Tensor, layout: dict) -> torch.Tensor:
    """(q, z, y, x) view of a flat copy of the grid storage, x counted from the first ghost cell"""
    st = tuple(int(s) for s in layout["strides_qzyx"])
    shape = tuple(int(s) for s in layout["shape_qzyx"])
    off = int(layout["x_offset_cells"]) * st[3]
    return torch.as_strided(storage, shape, st, off)


class ExchangeCheck:
    """load a random field into a halo workload's grid and check an exchange against the model.

    field "random": drawn on the host by a torch generator, the whole global field on every
    rank (small grids); "hashed": `hashed_values`, each rank computes only its own block (any
    size, any rank count). The copies of the grid and the model live on `device` ("cpu", or
    "cuda:N" for large grids)."""

    def __init__(self, halo, seed: int = 0, sentinel: float = -2.5, device="cpu",
                 field: str = "random"):
        if field not in ("random", "hashed"):
            raise ValueError(f"field must be random or hashed (got {field!r})")
        self.halo = halo
        self.device = torch.device(device)
        self.kind = field
        self.seed = seed
        self.layout = halo.layout()
        self.g = int(self.layout["ghost"])
        nq, Z, Y, X = (int(s) for s in self.layout["shape_qzyx"])
        self.nq = nq
        self.n_zyx = (Z - 2 * self.g, Y - 2 * self.g, X - 2 * self.g)
        cx, cy, cz = halo.coords()
        px, py, pz = halo.rank_grid()
        self.coords_zyx = (cz, cy, cx)
        self.extent = tuple(c * n for c, n in zip((pz, py, px), self.n_zyx))
        self.field = (global_field(nq, self.extent, seed).to(self.device) if field == "random"
                      else None)
        self.sentinel = sentinel
        self.neighbors = int(halo.args.neighbors)

    def load(self):
        """interior = this rank's slice of the field, every ghost cell = sentinel"""
        storage = torch.zeros(self.halo.grid_elems(), dtype=torch.float64, device=self.device)
        self._sync()
        self.halo.read_grid(storage.data_ptr())
        view = logical_view(storage, self.layout)
        view.fill_(self.sentinel)
        g = self.g
        if self.field is not None:
            sl = [slice(None)] + [slice(c * n, (c + 1) * n)
                                  for c, n in zip(self.coords_zyx, self.n_zyx)]
            view[:, g:-g, g:-g, g:-g] = self.field[tuple(sl)]
        else:
            view[:, g:-g, g:-g, g:-g] = self._hashed()[:, g:-g, g:-g, g:-g]
        self.before = view.clone()
        self._sync()  # torch's writes land before the copy (the copy runs on the null stream)
        self.halo.write_grid(storage.data_ptr())

    def mismatches(self) -> dict:
        """cells that differ from the model, by ghost class (0 interior ... 3 corner). Call it
        once the exchange has completed on the device (`HipRuntime.device_sync()`): the copy runs
        on the null stream, which does not wait for the runtime's non-blocking streams"""
        storage = torch.empty(self.halo.grid_elems(), dtype=torch.float64, device=self.device)
        self._sync()
        self.halo.read_grid(storage.data_ptr())
        got = logical_view(storage, self.layout)
        if self.field is not None:
            want = expected_block(self.field, self.coords_zyx, self.n_zyx, self.g,
                                  self.neighbors, self.before)
        else:
            want = self._hashed()
            if self.neighbors == 6:
                keep = (ghost_class(self.n_zyx, self.g) >= 2).to(self.device).expand_as(want)
                want[keep] = self.before[keep]
        bad = got != want
        cls = ghost_class(self.n_zyx, self.g).to(self.device).expand_as(bad)
        return {k: int(bad[cls == k].sum()) for k in range(4)}

    def _hashed(self) -> torch.Tensor:
        return hashed_block(self.nq, self.coords_zyx, self.n_zyx, self.extent, self.g, self.seed,
                            self.device)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def check_prepared(halo, rt, ctrl, device: int, seed: int = 20261) -> dict:
    """One exchange of the schedule prepared on `rt`, from a hashed field, every cell of every
    rank's padded block compared with the model on `device`; bad cells summed over ranks by
    ghost class (interior, face, edge, corner). Collective: every rank calls it together. The
    grid holds the hashed field afterwards (re-initialize it before a device-side check)."""
    torch.cuda.set_device(device)
    rt.device_sync()
    ctrl.barrier()
    chk = ExchangeCheck(halo, seed=seed, device=f"cuda:{device}", field="hashed")
    chk.load()
    ctrl.barrier()  # every rank's field is in place before any peer's puts land
    rt.run(1)
    rt.device_sync()
    ctrl.barrier()
    m = chk.mismatches()
    del chk
    torch.cuda.empty_cache()
    by = [int(v) for v in ctrl.allreduce_sum([float(m[k]) for k in range(4)])]
    return {"bad_cells": sum(by), "by_ghost_class": by, "field": "hashed"}
