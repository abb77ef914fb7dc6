"""Isolated kernel bandwidth microbenchmarks for the halo / copy kernels (MI355X).

python scripts/kbench.py [--n 512] [--neighbors 26] [--reps 50] [--order xyzq]
                         [--ghost-align -2] [--widen-ab]
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
    ap.add_argument("--ghost-align", type=int, default=-2,
                    help="HaloConfig.ghost_align: -2 auto (16), -1 x = 0 at the row start, 8, 16")
    ap.add_argument("--widen-ab", action="store_true",
                    help="only the 26-box unpack with the widened rows off / on, interleaved")
    ap.add_argument("--grid-memory-ab", action="store_true",
                    help="only the 26-direction move, pack and unpack on a coarse- and a "
                         "fine-grained grid, interleaved")
    args = ap.parse_args()
    torch.zeros(1, device="cuda")
    cfg = dict(n=args.n, neighbors=args.neighbors, order=args.order, ghost_align=args.ghost_align)
    if args.grid_memory_ab:
        st = torch.cuda.current_stream().cuda_stream
        hs = {}
        for mem in (0, 1):
            c, _ = build_halo(HaloConfig(transport="copy", grid_memory=mem, **cfg), tz.SelfCtrl(), device=0)
            d, _ = build_halo(HaloConfig(transport="direct", grid_memory=mem, **cfg), tz.SelfCtrl(), device=0)
            hs[c.grid_memory()] = (c, d)
        dirs = list(range(hs["fine"][1].ndirs()))
        for rnd in range(3):
            for mem, (c, d) in hs.items():
                r = dict(op="grid_memory_ab", grid_memory=mem, round=rnd)
                r["direct_all_us"] = round(timeit(lambda: d.direct_group(dirs, st), max(5, args.reps // 5)), 3)
                r["pack_all_us"] = round(timeit(lambda: c.pack_all(st), max(5, args.reps // 5)), 3)
                r["unpack_all_us"] = round(timeit(lambda: c.unpack_all(st), max(5, args.reps // 5)), 3)
                print(json.dumps(r), flush=True)
        for mem, (c, d) in hs.items():
            d.init_grid()
            d.direct_group(dirs, st)
            torch.cuda.synchronize()
            print(json.dumps(dict(grid_memory=mem, check_grid=int(d.check_grid()))), flush=True)
        return
    h, _ = build_halo(HaloConfig(transport="copy", **cfg), tz.SelfCtrl(), device=0)
    print(json.dumps({"order": args.order, "grid_bytes": h.grid_elems() * 8,
                      "layout": h.layout()}), flush=True)
    st = torch.cuda.current_stream().cuda_stream
    if args.widen_ab:
        K = tz._tz.kernels
        tot = h.exchange_bytes()
        for rnd in range(3):
            for widen in (False, True):
                K.set_widen_unpack(widen)
                us = timeit(lambda: h.unpack_all(st), max(5, args.reps // 5))
                print(json.dumps(dict(op="unpack_all", widen=widen, round=rnd, us=round(us, 3),
                                      GBps=round(2 * tot / us / 1e3, 1))), flush=True)
        K.set_widen_unpack(True)
        return
    hd, _ = build_halo(HaloConfig(transport="direct", **cfg), tz.SelfCtrl(), device=0)
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
