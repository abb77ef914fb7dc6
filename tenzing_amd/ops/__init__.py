"""Torch-tensor front ends of the hand-written gfx950 kernels (``tenzing_amd._tz.kernels``) and
of the RCCL communication ops (``tenzing_amd.ops.comm``).

Every function checks device, dtype, contiguity and sizes on the host before launching (the
kernels index raw pointers), then launches on torch's current stream. They fail loudly when the
native extension or a GPU is missing; there is no silent PyTorch fallback.
"""
from . import comm  # noqa: F401
from .kernels import (  # noqa: F401
    box_pack,
    box_unpack,
    copy_,
    csr_spmv,
    gather,
    vector_add,
)
