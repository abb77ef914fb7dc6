"""Distributed row-partitioned CSR SpMV workload.

Reference config (tenzing-mcts/examples/spmv_run_strategy.cuh:44-68; tenzing-dfs/examples/
spmv.cu:86-117): m=150,000 rows, nnz = 10 m, band width m / ranks, f32 values / i32 indices,
2 streams; MCTS 300 iterations or DFS up to 15,000 sequences, 50 benchmark iterations.
"""
from __future__ import annotations

import dataclasses

from .. import _tz


@dataclasses.dataclass
class SpmvConfig:
    m: int = 150_000
    bw: int = 0        # 0 = m / ranks
    nnz: int = 0       # 0 = 10 m
    seed: int = 1
    compound: bool = True       # expandable CompoundOp (reference SpMV CompoundOp)
    kernel_choice: bool = True  # local SpMV kernel variants as a ChoiceOp
    form: str = "choice"        # split (y = yl + yr, reference) | accum (y = yl; y += yr) | choice
    library: str = "adaptive"   # rocSPARSE CSR algorithm added to the kernel ChoiceOp ("" = none)
    transport: str = "auto"     # x halo between ranks: rccl | ipc | auto (ChoiceOp over both)
    prefix: str = ""
    matrix: str = ""            # Matrix Market file of a square matrix instead of the band matrix
    # root: rank 0 builds / reads the matrix and sends each rank its rows, the ranks then ask
    # the owners for the x entries they need (the reference's setup); local: every rank builds
    # it all itself; auto: root with a control plane of several ranks
    distribute: str = "auto"

    def args(self, rank: int = 0, size: int = 1, device: int = -1) -> "_tz.SpmvArgs":
        a = _tz.SpmvArgs()
        a.m, a.bw, a.nnz, a.seed = self.m, self.bw, self.nnz, self.seed
        a.compound, a.kernel_choice, a.prefix = self.compound, self.kernel_choice, self.prefix
        a.form = self.form
        a.library = self.library
        a.transport = self.transport
        a.matrix = self.matrix
        a.distribute = self.distribute
        a.rank, a.size, a.device = rank, size, device
        return a


def build_spmv(cfg: SpmvConfig, ctrl=None, device: int = -1, setup: bool = True, graph=None):
    rank = ctrl.rank if ctrl is not None else 0
    size = ctrl.size if ctrl is not None else 1
    s = _tz.DistSpmv(cfg.args(rank, size, device), ctrl if size > 1 else None)
    if setup:
        s.setup(ctrl)
    g = graph if graph is not None else _tz.Graph()
    s.add_to_graph(g)
    return s, g
