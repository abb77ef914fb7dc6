"""Checked torch wrappers for the native kernels."""
from __future__ import annotations

import torch

from .. import _tz

K = _tz.kernels


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _box_extent(box: dict) -> int:
    return box["len"] * box["n1"] * box["n2"] * box["n3"]


def _box_span(box: dict) -> int:
    """largest grid element index touched + 1"""
    return (box["grid_off"] + (box["n1"] - 1) * box["s1"] + (box["n2"] - 1) * box["s2"]
            + (box["n3"] - 1) * box["s3"] + box["len"])


def box_pack(grid: torch.Tensor, box: dict, out: torch.Tensor | None = None) -> torch.Tensor:
    """Gather the box (rows of ``len`` contiguous f64 at ``grid_off + i1*s1 + i2*s2 + i3*s3``)
    into a dense buffer."""
    _check(grid, torch.float64, "grid")
    if _box_span(box) > grid.numel():
        raise IndexError("box exceeds grid")
    n = _box_extent(box)
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=grid.device)
    _check(out, torch.float64, "out")
    if out.numel() < n:
        raise ValueError("out too small")
    K.box_copy(grid.data_ptr(), dict(box, buf=out.data_ptr()), False, _stream())
    return out


def box_unpack(grid: torch.Tensor, box: dict, buf: torch.Tensor) -> torch.Tensor:
    _check(grid, torch.float64, "grid")
    _check(buf, torch.float64, "buf")
    if _box_span(box) > grid.numel():
        raise IndexError("box exceeds grid")
    if buf.numel() < _box_extent(box):
        raise ValueError("buf too small")
    K.box_copy(grid.data_ptr(), dict(box, buf=buf.data_ptr()), True, _stream())
    return grid


def csr_spmv(row_ptr: torch.Tensor, col_ind: torch.Tensor, val: torch.Tensor, x: torch.Tensor,
             y: torch.Tensor | None = None, lanes: int = 0, accumulate: bool = False) -> torch.Tensor:
    """y = A x (or y += A x) for CSR A with int32 indices and f32 values."""
    _check(row_ptr, torch.int32, "row_ptr")
    _check(col_ind, torch.int32, "col_ind")
    _check(val, torch.float32, "val")
    _check(x, torch.float32, "x")
    n = row_ptr.numel() - 1
    if col_ind.numel() != val.numel():
        raise ValueError("col_ind and val differ in length")
    if y is None:
        y = torch.zeros(n, dtype=torch.float32, device=x.device)
    _check(y, torch.float32, "y")
    if y.numel() < n:
        raise ValueError("y too small")
    if lanes not in (-1, 0, 1, 2, 4, 8, 16, 32, 64):
        raise ValueError("lanes must be a power of two <= 64 (or -1: CSR-stream kernel)")
    K.csr_spmv(n, row_ptr.data_ptr(), col_ind.data_ptr(), val.data_ptr(), x.data_ptr(),
               y.data_ptr(), lanes, accumulate, _stream())
    return y


def gather(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    _check(src, torch.float32, "src")
    _check(idx, torch.int32, "idx")
    out = torch.empty(idx.numel(), dtype=torch.float32, device=src.device)
    K.gather_f32(idx.numel(), src.data_ptr(), idx.data_ptr(), out.data_ptr(), _stream())
    return out


def vector_add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    _check(a, torch.float32, "a")
    _check(b, torch.float32, "b")
    if a.numel() != b.numel():
        raise ValueError("size mismatch")
    y = torch.empty_like(a)
    K.vector_add_f32(a.numel(), a.data_ptr(), b.data_ptr(), y.data_ptr(), _stream())
    return y


def copy_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    if not (dst.is_cuda and src.is_cuda and dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("contiguous GPU tensors required")
    nb = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nb:
        raise ValueError("dst too small")
    K.copy_bytes(dst.data_ptr(), src.data_ptr(), nb, _stream())
    return dst
