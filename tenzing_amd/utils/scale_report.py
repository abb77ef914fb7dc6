"""A table of bench records at several GPU counts: what each run measured against what its own
link probes say the exchange could take.

``python -m tenzing_amd.utils.scale_report FILE [FILE ...]``: every bench record in the files
(the JSON lines ``bench.py`` prints, one record, or any JSON nesting records, such as a driver's
scaling file), one row per record, sorted by GPU count:

* ``ms``: the record's value (ms per exchange, max over ranks);
* ``busiest_link_ms``: the bytes the busiest link of the rank grid carries per exchange at the
  rate one kernel put reached over one link in the run's own probe (``link_probe``): a floor
  for any schedule that sends each face over its own link once;
* ``ms / link floor``: how far above that floor the run ended;
* the transport of the timed schedule, the search's wall-clock, and the model check's rank
  correlation (``model_check``).

Weak-scaling efficiency (the N=1 time over the N-GPU time) is printed for reference; the driver
computes its own from the same values.

Reference: the drivers print per-rank timings only (src/benchmarker.cpp:83-167); the reference
has no cross-run report.
"""
from __future__ import annotations

import json


def records(paths) -> list:
    """Every dict with a ``metric`` and a ``value`` (a bench record) in the files."""
    out = []

    def walk(o):
        if isinstance(o, dict):
            if "metric" in o and "value" in o and "n_gpus" in o:
                out.append(o)
                return
            o = list(o.values())
        if isinstance(o, list):
            for v in o:
                walk(v)

    for p in paths:
        text = open(p).read()
        try:
            walk(json.loads(text))
        except ValueError:
            lines = [json.loads(x) for x in text.splitlines() if x.strip().startswith("{")]
            # a bench run prints partial lines before the final one: keep the last per run
            finals = [d for d in lines if not d.get("partial")] or lines[-1:]
            walk(finals)
    return out


def rows(recs) -> list:
    base = {}
    for r in recs:
        if int(r.get("n_gpus") or 1) == 1 and r.get("value"):
            base.setdefault("ms", float(r["value"]))
    out = []
    for r in sorted(recs, key=lambda d: int(d.get("n_gpus") or 1)):
        n = int(r.get("n_gpus") or 1)
        ms = float(r["value"]) if r.get("value") is not None else None
        lp = r.get("link_probe") or {}
        floor = lp.get("busiest_link_at_probe_rate_ms")
        mc = r.get("model_check") or {}
        out.append({
            "n_gpus": n, "ms": ms, "partial": r.get("partial"),
            "bad_cells": r.get("verified_bad_cells"),
            "transport": r.get("schedule_transport"),
            "rank_grid": (r.get("config") or {}).get("rank_grid"),
            "busiest_link_ms": floor,
            "ms_over_link_floor": round(ms / floor, 2) if ms and floor else None,
            "put_GBps": (lp.get("GBps") or {}).get("put"),
            "search_wall_s": r.get("search_wall_s"),
            "model_spearman": mc.get("spearman"),
            "weak_efficiency": round(base["ms"] / ms, 3) if ms and "ms" in base else None,
        })
    return out


def _fmt(v):
    if v is None:
        return "-"
    if isinstance(v, float):
        return f"{v:.4g}"
    return str(v)


def _main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="python -m tenzing_amd.utils.scale_report")
    ap.add_argument("files", nargs="+")
    ap.add_argument("--json", action="store_true", help="one JSON line per row instead of a table")
    a = ap.parse_args(argv)
    rs = rows(records(a.files))
    if not rs:
        print("no bench records found")
        return 1
    if a.json:
        for r in rs:
            print(json.dumps(r))
        return 0
    cols = ["n_gpus", "ms", "partial", "bad_cells", "transport", "rank_grid", "busiest_link_ms",
            "ms_over_link_floor", "put_GBps", "search_wall_s", "model_spearman", "weak_efficiency"]
    table = [[_fmt(r[c]) for c in cols] for r in rs]
    w = [max(len(c), *(len(t[i]) for t in table)) for i, c in enumerate(cols)]
    print("  ".join(c.ljust(w[i]) for i, c in enumerate(cols)))
    for t in table:
        print("  ".join(x.ljust(w[i]) for i, x in enumerate(t)))
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
