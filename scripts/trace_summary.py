#!/usr/bin/env python3
"""Summarize a rocprofv3 kernel trace (CSV) into a small text report that can be committed.

The report covers the LAST `--last` dispatches (the timed loop of bench.py ends the run):
per-kernel medians, a timeline with the hardware queue of every dispatch and the idle gaps
between consecutive dispatches, and the total window. `--delete` removes the (large) CSV
afterwards so it does not travel back from the GPU box.

  python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --last 200 \
      --out gpurun_out/prof/timeline.txt --delete
"""
from __future__ import annotations

import argparse
import csv
import os
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:48]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=200)
    ap.add_argument("--timeline", type=int, default=60, help="timeline rows to print")
    ap.add_argument("--out", default="")
    ap.add_argument("--delete", action="store_true")
    a = ap.parse_args()

    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         short(r["Kernel_Name"]), int(r["Grid_Size_X"])))
    rows.sort()
    total = len(rows)
    rows = rows[-a.last:]
    lines = [f"dispatches in trace: {total}; summarizing the last {len(rows)}"]
    if rows:
        t0 = rows[0][0]
        per = defaultdict(list)
        for s, e, q, n, g in rows:
            per[(n, g)].append((e - s) / 1e3)
        lines.append(f"{'kernel':48s} {'grid':>9s} {'n':>5s} {'med us':>8s} {'sum us':>9s}")
        for (n, g), d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            lines.append(f"{n:48s} {g:9d} {len(d):5d} {statistics.median(d):8.2f} {sum(d):9.1f}")
        window = (rows[-1][1] - t0) / 1e3
        busy = 0.0
        cur_s, cur_e = rows[0][0], rows[0][1]
        for s, e, *_ in rows[1:]:
            if s > cur_e:
                busy += (cur_e - cur_s)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        busy /= 1e3
        lines.append(f"window {window:.1f} us, GPU busy (union of kernels) {busy:.1f} us "
                     f"({100 * busy / max(window, 1e-9):.1f}%), idle {window - busy:.1f} us")
        lines.append(f"{'kernel':48s} {'grid':>9s} {'q':>3s} {'start':>9s} {'end':>9s} "
                     f"{'dur':>7s} {'gap':>7s}")
        last_end = None
        for s, e, q, n, g in rows[-a.timeline:]:
            gap = "" if last_end is None else f"{(s - last_end) / 1e3:7.1f}"
            lines.append(f"{n:48s} {g:9d} {q:3d} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} "
                         f"{(e - s) / 1e3:7.1f} {gap:>7s}")
            last_end = e if last_end is None else max(last_end, e)
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    if a.delete:
        os.remove(a.trace)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
