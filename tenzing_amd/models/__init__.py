"""Workload "model families" (the reference's op libraries): 3-D halo exchange, distributed CSR
SpMV, and their fused graph."""
from .halo import HaloConfig, build_halo  # noqa: F401
from .spmv import SpmvConfig, build_spmv  # noqa: F401
from .fused import build_fused  # noqa: F401
