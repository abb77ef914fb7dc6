"""tenzing_amd — MI355X-native schedule search for multi-GPU HIP + RCCL programs.

A program is a DAG of operations (HIP kernels, RCCL transfers, host steps). The engine turns
"issue order x HIP-stream assignment x kernel variant x event-synchronization placement" into a
sequential decision problem, explores it with DFS or Monte-Carlo tree search, and benchmarks every
candidate schedule on the GPUs (eagerly or as a captured hipGraph). Same capabilities as
sandialabs/tenzing; see SURVEY.md for the parity map.

The search engine, runtime, kernels and transports are native (``tenzing_amd._tz``); this package
adds Python-side configuration, process bootstrap and analysis.
"""
from __future__ import annotations

import importlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


def _load_torch_first():
    """The extension and PyTorch-ROCm must share ONE HIP runtime in a process: both link
    libamdhip64.so.7 / librccl.so.1 by soname, so whichever is loaded first serves both. Loading
    torch first makes the process use torch's bundled runtime, so torch tensors, streams and our
    schedules interoperate (torch ops on our streams fail with invalid-argument otherwise)."""
    if os.environ.get("TZ_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _load_native():
    _load_torch_first()
    try:
        return importlib.import_module("tenzing_amd._tz")
    except ImportError as first:
        if os.environ.get("TZ_NO_AUTOBUILD"):
            raise
        from . import _build

        sys.stderr.write("tenzing_amd: native extension missing, building (gfx950)...\n")
        try:
            _build.build()
        except Exception as e:  # pragma: no cover - surfaced to the user
            raise ImportError(f"tenzing_amd native extension could not be built: {e}") from first
        importlib.invalidate_caches()
        return importlib.import_module("tenzing_amd._tz")


_tz = _load_native()

from ._tz import (  # noqa: E402,F401
    AllGatherOp,
    AllReduceOp,
    AlltoallvOp,
    BenchOpts,
    BenchResult,
    BoundGpuOp,
    BroadcastOp,
    BusyKernelOp,
    CommOp,
    CsvBenchmarker,
    Ctrl,
    DfsOpts,
    DistSpmv,
    EmptyKernelOp,
    EmpiricalBenchmarker,
    EventRecord,
    EventSync,
    ExecMode,
    Finish,
    Graph,
    HaloArgs,
    HaloExchange,
    HipRuntime,
    HostFuncOp,
    HostExecutor,
    MctsOpts,
    NoOp,
    OpBase,
    OpIndex,
    Platform,
    PyBenchmarker,
    PyCpuOp,
    PyGpuOp,
    RcclComm,
    ReduceScatterOp,
    RunDeadline,
    SelfCtrl,
    SendRecvOp,
    Sequence,
    SimBenchmarker,
    SimExecutor,
    SimGpuOp,
    SimParams,
    SleepOp,
    SpmvArgs,
    Start,
    State,
    StaticChoiceOp,
    StaticCompoundOp,
    StreamSync,
    StreamWait,
    StreamWaitEvent,
    TcpCtrl,
    TzError,
    agree_dead_domains,
    dead_domains,
    dfs_explore,
    domain_dead,
    enable_roctx,
    get_all_sequences,
    hip_device_count,
    mark_domain_dead,
    mcts_explore,
    random_rollout,
    remove_redundant_syncs,
    resolve_graph,
    revive_domains,
    strategy_names,
    verify,
)

from .search import run, search  # noqa: E402,F401


def _apply_env_options():
    """Process-wide runtime options from the environment, for programs (bench.py, the CLIs'
    subprocess tests) that cannot call the setters themselves: TZ_GRAPH_CAPTURE (schedule |
    child | auto) and TZ_PAD_STREAMS (streams a runtime owns at least). The native library reads
    neither: both are plain runtime options (``_tz.set_graph_capture``,
    ``_tz.set_default_pad_streams``) that one process can flip both ways."""
    v = os.environ.get("TZ_GRAPH_CAPTURE", "")
    if v:
        _tz.set_graph_capture(v)
    v = os.environ.get("TZ_PAD_STREAMS", "")
    if v:
        _tz.set_default_pad_streams(max(0, int(v)))


_apply_env_options()

__version__ = _tz.version()

NATIVE_PATH = _tz.__file__


def native_loaded() -> str:
    """Path of the loaded native extension (raises if the HIP path is not available)."""
    return NATIVE_PATH
