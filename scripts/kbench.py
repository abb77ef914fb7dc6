"""Isolated kernel bandwidth microbenchmarks for the halo / copy kernels (MI355X).

python scripts/kbench.py [--n 512] [--neighbors 26] [--reps 50]
Prints one JSON line per measurement: op, bytes moved (read+write), us, GB/s.
Interleaves variants in one process (methodology rule: A/B in one process).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def timeit(fn, reps):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--neighbors", type=int, default=26)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--order", default="xyzq")
    args = ap.parse_args()
    torch.zeros(1, device="cuda")
    h, _ = build_halo(HaloConfig(n=args.n, neighbors=args.neighbors, order=args.order,
                                 transport="copy"), tz.SelfCtrl(), device=0)
    hd, _ = build_halo(HaloConfig(n=args.n, neighbors=args.neighbors, order=args.order,
                                  transport="direct"), tz.SelfCtrl(), device=0)
    print(json.dumps({"order": args.order, "grid_bytes": h.grid_elems() * 8}), flush=True)
    st = torch.cuda.current_stream().cuda_stream
    out = []

    def rec(op, nbytes, us, **kw):
        r = dict(op=op, bytes=nbytes, us=round(us, 3), GBps=round(nbytes / us / 1e3, 1), **kw)
        print(json.dumps(r), flush=True)
        out.append(r)

    seen = set()
    for i in range(h.ndirs()):
        d = h.dir(i)
        kind = ("face" if sum(map(abs, d)) == 1 else "edge" if sum(map(abs, d)) == 2 else "corner")
        key = (kind, tuple(abs(x) for x in d))
        if key in seen:
            continue
        seen.add(key)
        nb = h.box_elems(i) * 8
        rec("pack", 2 * nb, timeit(lambda: h.pack(i, st), args.reps), dir=h.dir_name(i), kind=kind)
        rec("unpack", 2 * nb, timeit(lambda: h.unpack(h.opposite(i), st), args.reps), dir=h.dir_name(i), kind=kind)
        rec("shift", 2 * nb, timeit(lambda: h.shift(i, st), args.reps), dir=h.dir_name(i), kind=kind)
        rec("direct", 2 * nb, timeit(lambda: hd.direct(i, st), args.reps), dir=h.dir_name(i), kind=kind)
    tot = h.exchange_bytes()
    faces = [i for i in range(h.ndirs()) if sum(map(abs, h.dir(i))) == 1]
    small = [i for i in range(h.ndirs()) if sum(map(abs, h.dir(i))) > 1]
    fb = sum(h.box_elems(i) for i in faces) * 8
    rec("direct_all", 2 * tot, timeit(lambda: hd.direct_group(list(range(h.ndirs())), st), max(5, args.reps // 5)))
    rec("direct_faces", 2 * fb, timeit(lambda: hd.direct_group(faces, st), max(5, args.reps // 5)))
    if small:
        rec("direct_small", 2 * (tot - fb), timeit(lambda: hd.direct_group(small, st), args.reps))
    rec("pack_all", 2 * tot, timeit(lambda: h.pack_all(st), max(5, args.reps // 5)))
    rec("unpack_all", 2 * tot, timeit(lambda: h.unpack_all(st), max(5, args.reps // 5)))
    rec("shift_all", 2 * tot, timeit(lambda: h.shift_all(st), max(5, args.reps // 5)))
    # reference copies of a face-sized buffer
    nb = h.box_elems(0) * 8
    x = torch.empty(nb // 4, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    rec("torch_copy_face", 2 * nb, timeit(lambda: y.copy_(x), args.reps))
    rec("tz_copy_face", 2 * nb, timeit(lambda: tz._tz.kernels.copy_bytes(y.data_ptr(), x.data_ptr(), nb, st), args.reps))
    big = 1 << 30
    X = torch.empty(big // 4, dtype=torch.float32, device="cuda")
    Y = torch.empty_like(X)
    rec("tz_copy_1GiB", 2 * big, timeit(lambda: tz._tz.kernels.copy_bytes(Y.data_ptr(), X.data_ptr(), big, st), 10))
    rec("torch_copy_1GiB", 2 * big, timeit(lambda: Y.copy_(X), 10))
    rec("empty_kernel", 0, timeit(lambda: tz._tz.kernels.empty(st), 200))


if __name__ == "__main__":
    main()
