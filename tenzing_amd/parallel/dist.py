"""Multi-process bootstrap.

One process per GPU (``torchrun --nproc-per-node N``; RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT from the environment). The control plane is the native TCP star
(``tenzing_amd._tz.TcpCtrl``) and needs nothing from torch: rank 0 listens on the control port
(``TZ_CTRL_PORT``, default MASTER_PORT + 1: torchrun's agent already serves its own store on
MASTER_PORT; if another program holds it, the next of ``TZ_CTRL_PORTS`` = 8 candidates) and every
other rank connects to MASTER_ADDR with a handshake that only this job's rank 0 answers. So a multi-rank run
can use the system ROCm runtime (``TZ_NO_TORCH=1``) as well as torch's bundled one.
``TZ_CTRL_BOOTSTRAP=torch`` restores the old path (one gloo broadcast of an ephemeral port). RCCL
communicators for the data plane are created later by the workloads, with their unique ids
broadcast over that control plane.

Processes started by an MPI launcher instead (``mpirun -n 8 python bench.py``, the reference's
launch model) use ``MpiCtrl``: the control collectives then run over MPI_COMM_WORLD (host MPI,
opened at run time), and the node-local rank the launcher exports picks the GPU.

Reference: MPI_Init + MPI_COMM_WORLD everywhere (tenzing-mcts/examples/halo_min_time.cu:11,
spmv_run_strategy.cuh:81-90 rank -> device = rank % ndev).
"""
from __future__ import annotations

import dataclasses
import os

from .. import _tz


@dataclasses.dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500


def _mpi_launched() -> bool:
    return "WORLD_SIZE" not in os.environ and _tz.MpiCtrl.launched()


def env() -> DistEnv:
    if _mpi_launched():
        e = os.environ
        rank = int(e.get("PMI_RANK", e.get("PMIX_RANK", e.get("MV2_COMM_WORLD_RANK", 0))))
        world = _tz.MpiCtrl.launcher_size()
        local = _tz.MpiCtrl.launcher_local_rank()
        return DistEnv(rank, world, local if local >= 0 else rank)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return DistEnv(rank, world, local, os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   int(os.environ.get("MASTER_PORT", 29500)))


def init_ctrl(rank: int | None = None, world: int | None = None, master_addr: str | None = None,
              timeout_s: float = 300.0, backend: str = "auto") -> "_tz.Ctrl":
    """Create the native control plane for this process (SelfCtrl for a single process).

    backend: "tcp" (torchrun-style RANK / WORLD_SIZE rendezvous), "mpi" (MPI_COMM_WORLD) or
    "auto" (mpi when an MPI launcher started this process and WORLD_SIZE is unset)."""
    if backend not in ("auto", "tcp", "mpi"):
        raise ValueError(f"backend must be auto, tcp or mpi (got {backend!r})")
    if backend == "mpi" or (backend == "auto" and _mpi_launched()):
        ctrl = _tz.MpiCtrl()
        _tz.set_log_rank(ctrl.rank)
        return ctrl
    e = env()
    rank = e.rank if rank is None else rank
    world = e.world if world is None else world
    _tz.set_log_rank(rank)
    if world == 1:
        return _tz.SelfCtrl()
    how = os.environ.get("TZ_CTRL_BOOTSTRAP", "tcp")
    if how not in ("tcp", "torch"):
        raise ValueError(f"TZ_CTRL_BOOTSTRAP must be tcp or torch (got {how!r})")
    ctrl = _tz.TcpCtrl(rank, world)
    host = master_addr or e.master_addr
    if how == "tcp":
        port = int(os.environ.get("TZ_CTRL_PORT", e.master_port + 1))
        # rank 0 takes the first free one of TZ_CTRL_PORTS candidate ports from there
        ctrl.rendezvous(host, port, timeout_s, int(os.environ.get("TZ_CTRL_PORTS", "8")))
        return ctrl
    import datetime

    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    port = ctrl.listen(0) if rank == 0 else 0
    box = [port]
    dist.broadcast_object_list(box, src=0)
    ctrl.connect(host, int(box[0]), timeout_s)
    return ctrl


def select_device(local_rank: int | None = None) -> int:
    """Bind this process to GPU ``local_rank % device_count`` (-1 when no GPU is visible)."""
    n = _tz.hip_device_count()
    if n == 0:
        return -1
    lr = env().local_rank if local_rank is None else local_rank
    return lr % n


def init(timeout_s: float = 300.0):
    """(ctrl, device) for this process.

    ``TZ_RCCL_LOOPBACK=1`` (tests on one GPU): RCCL refuses two ranks of one host on one device,
    so each rank gets a host id of its own (``NCCL_HOSTID``) and looks like a node of its own to
    RCCL; the ranks' communicators then connect through RCCL's network transport (sockets over
    ``lo``). Slow, but every RCCL code path runs across real rank boundaries."""
    ctrl = init_ctrl(timeout_s=timeout_s)
    if os.environ.get("TZ_RCCL_LOOPBACK") == "1" and ctrl.size > 1:
        os.environ.setdefault("NCCL_HOSTID", f"tz-loopback-rank{ctrl.rank}")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    return ctrl, select_device()
