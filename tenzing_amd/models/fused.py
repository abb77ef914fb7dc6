"""Distributed SpMV + halo exchange in one graph (BASELINE.json config 5: the largest decision
tree — both workloads' ops compete for the same streams)."""
from __future__ import annotations

import dataclasses

from .. import _tz
from .halo import HaloConfig, build_halo
from .spmv import SpmvConfig, build_spmv


def build_fused(halo_cfg: HaloConfig, spmv_cfg: SpmvConfig, ctrl=None, device: int = -1,
                setup: bool = True):
    g = _tz.Graph()
    h, _ = build_halo(halo_cfg, ctrl, device, setup, g)
    sp = dataclasses.replace(spmv_cfg, prefix=spmv_cfg.prefix or "spmv_")
    s, _ = build_spmv(sp, ctrl, device, setup, g)
    return h, s, g
