"""Torch-tensor front ends of the RCCL communication ops (``tenzing_amd._tz.SendRecvOp`` ...).

The reference's user-level communication ops are host-issued MPI requests
(include/tenzing/mpi/ops_mpi.hpp:17-192: ``Isend``, ``Irecv``, ``Ialltoallv``, ``Wait``,
``OwningWaitall``, ``MultiWait``). Here each transfer is a stream-bound graph op: the search
assigns it a HIP stream like a kernel, and its completion is ordered by the synchronizer's event
edges, so there is no separate wait op. Each function checks the tensors on the host (GPU,
contiguous, one dtype, sizes that match the collective) and returns an op whose lifetime keeps
the tensors alive.

``comms`` is one ``RcclComm`` or a list of them. An op bound to logical stream ``k`` uses
``comms[k % len(comms)]``; pass one communicator per stream
(``tz._tz.make_rccl_comms(ctrl, device, n_streams)``) so that no communicator is driven from two
streams at once.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import torch

from .. import _tz

DTYPES = {
    torch.float32: 0,
    torch.float64: 1,
    torch.int32: 2,
    torch.float16: 3,
    torch.bfloat16: 4,
    torch.int64: 5,
    torch.uint8: 6,
}
REDUCTIONS = {"sum": 0, "prod": 1, "max": 2, "min": 3}


def _comms(comms) -> list:
    cs = [comms] if isinstance(comms, _tz.RcclComm) else list(comms)
    if not cs:
        raise ValueError("at least one communicator is needed")
    return cs


def _check(t: torch.Tensor, name: str) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.dtype not in DTYPES:
        raise TypeError(f"{name}: unsupported dtype {t.dtype}")
    return DTYPES[t.dtype]


def _same_dtype(ts: Iterable[torch.Tensor]) -> int:
    codes = {_check(t, f"tensor {i}") for i, t in enumerate(ts)}
    if len(codes) != 1:
        raise TypeError("all tensors of one op must share a dtype")
    return codes.pop()


def _red(op: str) -> int:
    try:
        return REDUCTIONS[op]
    except KeyError:
        raise ValueError(f"reduction must be one of {sorted(REDUCTIONS)}") from None


def send_recv(name: str, comms, send: torch.Tensor | None, send_peer: int,
              recv: torch.Tensor | None, recv_peer: int):
    """Send ``send`` to ``send_peer`` and receive ``recv`` from ``recv_peer`` in one group
    (either side may be None)."""
    ts = [t for t in (send, recv) if t is not None]
    if not ts:
        raise ValueError("send_recv needs a send or a receive tensor")
    dt = _same_dtype(ts)
    return _tz.SendRecvOp(name, _comms(comms),
                          send.data_ptr() if send is not None else 0,
                          send.numel() if send is not None else 0, send_peer,
                          recv.data_ptr() if recv is not None else 0,
                          recv.numel() if recv is not None else 0, recv_peer, dt,
                          keep=tuple(ts))


def alltoallv(name: str, comms, sends: Sequence[tuple[torch.Tensor, int]],
              recvs: Sequence[tuple[torch.Tensor, int]]):
    """One group of sends ``[(tensor, peer)]`` and receives ``[(tensor, peer)]`` (the
    reference's ``Ialltoallv`` with per-peer buffers)."""
    ts = [t for t, _ in sends] + [t for t, _ in recvs]
    if not ts:
        raise ValueError("alltoallv needs at least one transfer")
    dt = _same_dtype(ts)
    xs = [(t.data_ptr(), t.numel(), p, 0, 0, -1) for t, p in sends]
    xs += [(0, 0, -1, t.data_ptr(), t.numel(), p) for t, p in recvs]
    return _tz.AlltoallvOp(name, _comms(comms), xs, dt, keep=tuple(ts))


def all_reduce(name: str, comms, tensor: torch.Tensor, out: torch.Tensor | None = None,
               op: str = "sum"):
    """``out = reduce(tensor over ranks)``; in place when ``out`` is None."""
    out = tensor if out is None else out
    dt = _same_dtype([tensor, out])
    if out.numel() != tensor.numel():
        raise ValueError("all_reduce: out must have as many elements as tensor")
    return _tz.AllReduceOp(name, _comms(comms), tensor.data_ptr(), out.data_ptr(), tensor.numel(),
                           dt, _red(op), keep=(tensor, out))


def all_gather(name: str, comms, tensor: torch.Tensor, out: torch.Tensor):
    """``out`` = every rank's ``tensor``, rank-major (``out.numel() == size * tensor.numel()``)."""
    cs = _comms(comms)
    dt = _same_dtype([tensor, out])
    if out.numel() != cs[0].size * tensor.numel():
        raise ValueError("all_gather: out must hold size * tensor.numel() elements")
    return _tz.AllGatherOp(name, cs, tensor.data_ptr(), out.data_ptr(), tensor.numel(), dt,
                           keep=(tensor, out))


def reduce_scatter(name: str, comms, tensor: torch.Tensor, out: torch.Tensor, op: str = "sum"):
    """Rank r gets the reduction of block r of ``tensor`` (``tensor.numel() == size * out.numel()``)."""
    cs = _comms(comms)
    dt = _same_dtype([tensor, out])
    if tensor.numel() != cs[0].size * out.numel():
        raise ValueError("reduce_scatter: tensor must hold size * out.numel() elements")
    return _tz.ReduceScatterOp(name, cs, tensor.data_ptr(), out.data_ptr(), out.numel(), dt,
                               _red(op), keep=(tensor, out))


def broadcast(name: str, comms, tensor: torch.Tensor, root: int = 0,
              out: torch.Tensor | None = None):
    """Root's ``tensor`` lands in every rank's ``out`` (in place when ``out`` is None)."""
    out = tensor if out is None else out
    dt = _same_dtype([tensor, out])
    if out.numel() != tensor.numel():
        raise ValueError("broadcast: out must have as many elements as tensor")
    return _tz.BroadcastOp(name, _comms(comms), tensor.data_ptr(), out.data_ptr(), tensor.numel(),
                           root, dt, keep=(tensor, out))
