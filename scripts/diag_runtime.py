"""Diagnostics: which HIP runtime / RCCL got loaded, and whether our runtime initializes.

usage: python scripts/diag_runtime.py [torch-first|native-first]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
if order == "torch-first":
    import torch

    torch.zeros(1, device="cuda")
import tenzing_amd as tz  # noqa: E402

maps = open("/proc/self/maps").read().splitlines()
libs = sorted({l.split()[-1] for l in maps if ("amdhip64" in l or "rccl" in l or "hsa-runtime" in l)})
print("order:", order, "libs:", libs, flush=True)
print("devices:", tz.hip_device_count(), flush=True)
rt = tz.HipRuntime(device=0, n_streams=2)
print("device:", rt.device_name(), flush=True)
