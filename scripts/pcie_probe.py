#!/usr/bin/env python3
"""What the GPU's PCIe link to the host carries, alone and in both directions at once.

Probe for a host-memory path beside xGMI: a share of a halo face could go GPU -> pinned host
memory -> peer GPU while the xGMI link carries the rest. Measures, for `--mb` MB transfers:
  * hipMemcpyAsync D2H, H2D, and both at once on two streams (copy engines);
  * a copy kernel (CUs) storing into pinned host memory, loading from it, and both at once;
  * a device-to-device copy of the same size, for reference.
One JSON line per measurement.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402

K = tz._tz.kernels


def timed(fn, streams, reps):
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    main = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ev0.record(main)
    for s in streams:
        s.wait_stream(main)
    for _ in range(reps):
        fn()
    for s in streams:
        main.wait_stream(s)
    ev1.record(main)
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=37.7)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n = int(a.mb * 1e6) // 16 * 16
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev3 = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    host2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def rec(name, secs, nbytes):
        print(json.dumps({"probe": name, "MB": nbytes / 1e6, "ms": secs * 1e3,
                          "GBps": nbytes / secs / 1e9}), flush=True)

    # copy engines
    def d2h():
        with torch.cuda.stream(s1):
            host.copy_(dev, non_blocking=True)

    def h2d():
        with torch.cuda.stream(s2):
            dev2.copy_(host2, non_blocking=True)

    rec("sdma_d2h", timed(d2h, [s1], a.reps), n)
    rec("sdma_h2d", timed(h2d, [s2], a.reps), n)
    rec("sdma_both", timed(lambda: (d2h(), h2d()), [s1, s2], a.reps), 2 * n)

    # CUs through the pinned mapping
    def k_d2h():
        K.copy_bytes(host.data_ptr(), dev.data_ptr(), n, s1.cuda_stream)

    def k_h2d():
        K.copy_bytes(dev2.data_ptr(), host2.data_ptr(), n, s2.cuda_stream)

    rec("kernel_store_to_host", timed(k_d2h, [s1], a.reps), n)
    rec("kernel_load_from_host", timed(k_h2d, [s2], a.reps), n)
    rec("kernel_both", timed(lambda: (k_d2h(), k_h2d()), [s1, s2], a.reps), 2 * n)

    def d2d():
        K.copy_bytes(dev3.data_ptr(), dev.data_ptr(), n, s1.cuda_stream)

    rec("kernel_d2d", timed(d2d, [s1], a.reps), n)
    torch.cuda.synchronize()
    del host, host2
    return 0


if __name__ == "__main__":
    sys.exit(main())
