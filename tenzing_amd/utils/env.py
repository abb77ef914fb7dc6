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
    """Pin this process to the GPU-local CPUs (no-op if unknown). Returns the CPU list used.

    Only the local CPUs this process may run on count. When fewer than 4 of them remain (a
    cpuset that holds other CPUs than the GPU's), the process stays unpinned: the HIP runtime's
    and RCCL's helper threads would otherwise share one or two CPUs with the search."""
    cpus = local_cpus(device)
    allowed = os.sched_getaffinity(0)
    cpus = [c for c in cpus if c in allowed]
    if len(cpus) < min(4, len(allowed)):
        return []
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def xgmi_topology() -> str:
    try:
        return subprocess.run(["rocm-smi", "--showtopotype"], capture_output=True, text=True,
                              timeout=20).stdout
    except Exception:  # noqa: BLE001
        return ""


def xgmi_topology_summary(timeout_s: float = 20.0):
    """The node's GPU link types as a compact matrix: {"gpus": N, "link_type": [[...]]}
    ("XGMI", "PCIE", "-" on the diagonal), from ``rocm-smi --showtopotype --json``; the raw
    table lines when the JSON form is unavailable; None without rocm-smi."""
    import json
    import re

    try:
        r = subprocess.run(["rocm-smi", "--showtopotype", "--json"], capture_output=True,
                           text=True, timeout=timeout_s)
    except Exception:  # noqa: BLE001
        return None
    try:
        doc = json.loads(r.stdout)
    except ValueError:
        lines = [ln.strip() for ln in (r.stdout or "").splitlines() if ln.strip()]
        return {"raw": lines[:24]} if lines else None
    pairs = {}
    n = 0
    for card, kv in doc.items():
        if not isinstance(kv, dict):
            continue
        for k, v in kv.items():
            m = re.search(r"between DRM devices (\d+) and (\d+)", k)
            if m:
                a, b = int(m.group(1)), int(m.group(2))
                pairs[(a, b)] = str(v)
                n = max(n, a + 1, b + 1)
    if not pairs:
        return {"raw_json_keys": list(doc)[:16]}
    mat = [["-" if i == j else pairs.get((i, j), pairs.get((j, i), "?")) for j in range(n)]
           for i in range(n)]
    return {"gpus": n, "link_type": mat,
            "xgmi_links": sum(1 for i in range(n) for j in range(i + 1, n) if mat[i][j] == "XGMI")}


def mapped_library(stem: str, maps: str | None = None) -> str | None:
    """Path of the shared library whose file name starts with ``stem`` (e.g. "libamdhip64")
    mapped into this process (``/proc/self/maps``), or None. Which copy a process maps decides
    what runs: torch's bundled runtime or the system ROCm's, whichever was loaded first."""
    if maps is None:
        maps = _read("/proc/self/maps")
    for line in maps.splitlines():
        parts = line.split(None, 5)
        if len(parts) == 6 and os.path.basename(parts[5]).startswith(stem + "."):
            return parts[5].strip()
    return None


def _hip_version_str(v: int) -> str | None:
    if v is None or v < 0:
        return None
    return f"{v // 10000000}.{(v // 100000) % 100}.{v % 100000}"


def _rccl_version_str(v: str) -> str:
    try:
        n = int(v)
    except ValueError:
        return v
    # NCCL_VERSION_CODE: major*10000 + minor*100 + patch (>= 2.9)
    return f"{n // 10000}.{(n // 100) % 100}.{n % 100}"


def runtime_libraries(maps: str | None = None) -> dict:
    """The HIP runtime and RCCL this process actually runs: mapped file + version reported by
    that library (not what /opt/rocm holds). Reference: src/reproduce.cpp:22-37 (version dump)."""
    return {
        "hip_runtime": {"path": mapped_library("libamdhip64", maps),
                        "version": _hip_version_str(_tz.hip_runtime_version())},
        "rccl_library": {"path": mapped_library("librccl", maps),
                         "version": _rccl_version_str(_tz.rccl_version())},
        "torch_loaded": "torch" in sys.modules,
    }


def env_report(device: int | None = None, topology: bool = False) -> dict:
    libs = runtime_libraries()
    r = {
        "tenzing_amd": _tz.version(),
        "python": sys.version.split()[0],
        "host": platform.node(),
        # what is installed under /opt/rocm; the process may run another copy (hip_runtime)
        "rocm_install": _read("/opt/rocm/.info/version"),
        "hip_runtime": libs["hip_runtime"],
        "rccl_library": libs["rccl_library"],
        "gpus": _tz.hip_device_count(),
    }
    torch = sys.modules.get("torch")  # reported when loaded; never imported just for this
    if torch is not None:
        r["torch"] = torch.__version__
        r["torch_hip"] = torch.version.hip
    if device is not None and r["gpus"] > 0:
        rt = _tz.HipRuntime(device=device, n_streams=1)
        r["device"] = rt.device_name()
        r["pci_bus_id"] = _tz.pci_bus_id(device)
        r["local_cpus"] = len(local_cpus(device))
    if topology:
        r["xgmi_topology"] = xgmi_topology()
        r["xgmi_topology_summary"] = xgmi_topology_summary()
    return r
