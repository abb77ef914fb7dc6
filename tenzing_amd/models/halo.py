"""3-D halo exchange workload.

Reference driver config (tenzing-mcts/examples/halo_run_strategy.hpp:42-49): nQ=3,
nX=nY=nZ=512, nGhost=3, XYZQ storage, 6 face neighbours, 2 streams. BASELINE.json's headline
adds the 27-point stencil (26 neighbours) and 4 streams per rank on 8 GPUs.

Graph per direction d: ``he_pack_<d> -> he_shift_<d> -> he_unpack_<-d>`` (rccl / copy
transports; see csrc/workloads/workloads.hpp for the RCCL design) or one pack-free
``he_direct_<d>`` box move straight into the neighbour's ghost region (direct transport, the
default on one rank). ``fuse`` groups directions into single launches / RCCL groups; "choice"
leaves the grouping to the search (ChoiceOps).
"""
from __future__ import annotations

import dataclasses

from .. import _tz


def ipc_grid_mode(value=None) -> int:
    """HaloArgs.ipc_grid: `value` if given, else TZ_IPC_GRID (1 grid, 0 receive buffers) from
    the environment, else -1 (auto). The environment is read here, where a config becomes
    native arguments, so one process can build both modes."""
    import os

    if value is None:
        v = os.environ.get("TZ_IPC_GRID", "")
        if v == "":
            return -1
        value = 1 if int(v) != 0 else 0
    value = int(value)
    if value not in (-1, 0, 1):
        raise ValueError(f"ipc_grid must be -1 (auto), 0 or 1 (got {value})")
    return value


@dataclasses.dataclass
class HaloConfig:
    n: int = 512          # interior cells per rank per axis (nX = nY = nZ)
    nq: int = 3           # quantities per cell
    ghost: int = 3        # ghost width
    neighbors: int = 26   # 6 = faces, 26 = faces + edges + corners (27-point stencil)
    order: str = "xyzq"   # storage order
    transport: str = "auto"  # rccl | copy | direct | auto (direct on 1 rank, else rccl)
    fuse: str = "none"    # none | pack | all | groups | choice
    comms: int = 0        # RCCL communicators (0 = one per direction)
    pitch_pad: int = 0    # extra row-pitch elements (multiple of 8; of 16 with line-aligned ghosts)
    rank_grid: tuple = ()  # (px, py, pz); () = reference rule (prime factors, smallest dim first)
    # x ghost runs aligned to 8 (sector) / 16 (line) elements, 0 = off, -1 = x = 0 at the row
    # start (the reference's layout), -2 = auto (16, line-aligned, in both orders)
    ghost_align: int = -2
    stencil: bool = False  # add a 7-point stencil (interior beside / shell after the exchange)
    # two-hop routing of a share of every face through the corner peer (2x2x2 rank grid, ipc
    # receive buffers): "auto" offers it to the search, "off", "force" (only transport)
    relay: str = "auto"
    # relayed shares offered (ChoiceOp): 0.2 balances the links when the forward waits for the
    # whole share, 0.25 is the link model's f* at equal link rates (parallel/linkmodel.relay_share)
    relay_fracs: tuple = (0.15, 0.2, 0.25)
    # a share of every face through node shared host memory over the GPUs' PCIe links, beside
    # the xGMI IPC put of the rest (ipc receive buffers): "auto" offers it, "off", "force"
    hostsplit: str = "auto"
    hostsplit_fracs: tuple = (0.1, 0.2, 0.3, 0.4)  # host shares offered (ChoiceOp)
    hostsplit_chunks: int = 1  # host share pipelined in this many chunks
    # IPC kernel puts with more workgroups per box, offered beside the default put: "auto"
    # (when peers sit on other devices), "on", "off"
    wide_puts: str = "auto"
    wide_put_blocks: int = 256
    # IPC puts into the peer's grid (1) or into receive buffers (0); None: the environment's
    # TZ_IPC_GRID if set, else auto (-1: the grid below 2 GiB)
    ipc_grid: int | None = None
    copy_puts: bool = True   # copy-engine puts offered (receive buffers only)
    copy_engines: int = 1    # copy-engine puts of one group spread over this many streams
    move_pairs: bool = True  # XYZQ x self-wrap moves as row pairs
    # grid memory: -1 auto (fine-grained in IPC grid mode, where peers store into it), 0 coarse,
    # 1 fine-grained
    grid_memory: int = -1
    # appended to the node identity: ranks of one node posing as several (tests); directions
    # whose neighbour is on another node go over RCCL, the rest keep IPC
    node_tag: str = ""

    def args(self, rank: int = 0, size: int = 1, device: int = -1) -> "_tz.HaloArgs":
        a = _tz.HaloArgs()
        a.nx = a.ny = a.nz = self.n
        a.nq = self.nq
        a.ghost = self.ghost
        a.neighbors = self.neighbors
        a.order = self.order
        a.transport = self.transport
        a.fuse = self.fuse
        a.comms = self.comms
        a.pitch_pad = self.pitch_pad
        a.ghost_align = self.ghost_align
        a.stencil = self.stencil
        a.relay = self.relay
        a.relay_fracs = [float(f) for f in self.relay_fracs]
        a.hostsplit = self.hostsplit
        a.hostsplit_fracs = [float(f) for f in self.hostsplit_fracs]
        a.hostsplit_chunks = int(self.hostsplit_chunks)
        a.wide_puts = self.wide_puts
        a.wide_put_blocks = int(self.wide_put_blocks)
        a.ipc_grid = ipc_grid_mode(self.ipc_grid)
        a.copy_puts = bool(self.copy_puts)
        a.copy_engines = int(self.copy_engines)
        a.move_pairs = bool(self.move_pairs)
        a.grid_memory = int(self.grid_memory)
        a.node_tag = str(self.node_tag)
        if self.rank_grid:
            a.px, a.py, a.pz = (int(v) for v in self.rank_grid)
        a.rank, a.size, a.device = rank, size, device
        return a


def build_halo(cfg: HaloConfig, ctrl=None, device: int = -1, setup: bool = True, graph=None):
    """Create the halo workload for this rank and add it to ``graph`` (new graph if None).

    ``setup=False`` builds the op graph only (no GPU needed: simulated / replayed searches).
    Returns (halo, graph)."""
    rank = ctrl.rank if ctrl is not None else 0
    size = ctrl.size if ctrl is not None else 1
    h = _tz.HaloExchange(cfg.args(rank, size, device))
    if setup:
        h.setup(ctrl)
    g = graph if graph is not None else _tz.Graph()
    h.add_to_graph(g)
    return h, g
