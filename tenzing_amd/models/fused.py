"""Distributed SpMV + halo exchange in one graph (BASELINE.json config 5: the largest decision
tree — both workloads' ops compete for the same streams).

On one rank (every halo direction a self move, no remote SpMV part) the graph also offers
horizontal fusion: one kernel launch that runs the 26-direction move and the SpMV's local
product at once, their workgroups interleaved (``_tz.move_spmv_op``, ``kern::box_move_spmv``).
The top-level ChoiceOp ``hs_launches`` picks between the two workloads' own ops (``hs_separate``,
everything the search otherwise decides) and that one launch with the ILP SpMV at 4 or 2 lanes
per row (``hs_onelaunch_i4`` / ``_i2``)."""
from __future__ import annotations

import dataclasses

from .. import _tz
from .halo import HaloConfig, build_halo
from .spmv import SpmvConfig, build_spmv

SPMV_ILP = 1000  # kern::kSpmvIlp: lanes = SPMV_ILP + lanes per row selects the ILP kernel


def build_fused(halo_cfg: HaloConfig, spmv_cfg: SpmvConfig, ctrl=None, device: int = -1,
                setup: bool = True, horizontal: bool = True):
    g = _tz.Graph()
    h, _ = build_halo(halo_cfg, ctrl, device, setup, g)
    sp = dataclasses.replace(spmv_cfg, prefix=spmv_cfg.prefix or "spmv_")
    s, _ = build_spmv(sp, ctrl, device, setup, g)
    size = ctrl.size if ctrl is not None else 1
    direct = [i for i in range(h.ndirs()) if h.is_direct(i)]
    if horizontal and size == 1 and len(direct) == h.ndirs() and not halo_cfg.stencil:
        alts = [_tz.StaticCompoundOp("hs_separate", g)]
        for w in (4, 2):
            alts.append(_tz.move_spmv_op(h, direct, s, f"hs_onelaunch_i{w}", SPMV_ILP + w, True))
        top = _tz.StaticChoiceOp("hs_launches", alts)
        g = _tz.Graph()
        g.start_then(top)
        g.then_finish(top)
    return h, s, g
