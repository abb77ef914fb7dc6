#!/usr/bin/env python3
"""How long does hipIpcOpenMemHandle take per allocation size (same device, two processes)?

  python scripts/ipc_probe.py export DIR &   python scripts/ipc_probe.py import DIR
"""
import ctypes
import os
import sys
import time

import torch  # loads torch's HIP runtime

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
SIZES_GB = [0.5, 1.0, 1.5, 1.9, 2.1, 3.0]


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(Handle), ctypes.c_void_p]


def main():
    mode, d = sys.argv[1], sys.argv[2]
    torch.zeros(1, device="cuda")
    if mode == "export":
        ptrs = []
        for gb in SIZES_GB:
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(int(gb * 2**30))) == 0
            h = Handle()
            assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
            ptrs.append(p)
            with open(os.path.join(d, f"h{gb}"), "wb") as f:
                f.write(bytes(h))
        open(os.path.join(d, "ready"), "w").close()
        while not os.path.exists(os.path.join(d, "done")):
            time.sleep(0.2)
        return
    while not os.path.exists(os.path.join(d, "ready")):
        time.sleep(0.2)
    for gb in SIZES_GB:
        h = Handle.from_buffer_copy(open(os.path.join(d, f"h{gb}"), "rb").read())
        p = ctypes.c_void_p()
        t0 = time.time()
        r = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
        print(f"{gb} GB: rc={r} {time.time() - t0:.2f} s", flush=True)
        if r == 0:
            hip.hipIpcCloseMemHandle(p)
    open(os.path.join(d, "done"), "w").close()


if __name__ == "__main__":
    main()
