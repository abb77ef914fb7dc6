"""Environment reporting and GPU-affine CPU binding.

* ``env_report()`` extends the reference's reproducibility dump (src/reproduce.cpp:22-37:
  version + hash + args) with ROCm / HIP / RCCL versions, GPU name and the xGMI link topology.
* ``bind_local_cpus(device)`` pins the calling process to the CPUs of the NUMA node its GPU hangs
  off (reference: src/numa.cpp ``bind_to_local_memory``, which is dead code there because its
  guard macro is never defined).
"""
from __future__ import annotations

import os
import platform
import subprocess
import sys

from .. import _tz


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def parse_cpulist(s: str) -> list[int]:
    cpus = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def local_cpus(device: int) -> list[int]:
    bus = _tz.pci_bus_id(device).lower()
    if not bus:
        return []
    return parse_cpulist(_read(f"/sys/bus/pci/devices/{bus}/local_cpulist"))


def bind_local_cpus(device: int) -> list[int]:
    """Pin this process to the GPU-local CPUs (no-op if unknown). Returns the CPU list used."""
    cpus = local_cpus(device)
    allowed = os.sched_getaffinity(0)
    cpus = [c for c in cpus if c in allowed]
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def xgmi_topology() -> str:
    try:
        return subprocess.run(["rocm-smi", "--showtopotype"], capture_output=True, text=True,
                              timeout=20).stdout
    except Exception:  # noqa: BLE001
        return ""


def env_report(device: int | None = None, topology: bool = False) -> dict:
    r = {
        "tenzing_amd": _tz.version(),
        "python": sys.version.split()[0],
        "host": platform.node(),
        "rocm": _read("/opt/rocm/.info/version"),
        "rccl": _tz.rccl_version(),
        "gpus": _tz.hip_device_count(),
    }
    try:
        import torch

        r["torch"] = torch.__version__
        r["torch_hip"] = torch.version.hip
    except Exception:  # noqa: BLE001
        pass
    if device is not None and r["gpus"] > 0:
        rt = _tz.HipRuntime(device=device, n_streams=1)
        r["device"] = rt.device_name()
        r["pci_bus_id"] = _tz.pci_bus_id(device)
        r["local_cpus"] = len(local_cpus(device))
    if topology:
        r["xgmi_topology"] = xgmi_topology()
    return r
