#!/usr/bin/env python3
"""Median counter value per (kernel, grid, counter) from rocprofv3 counter_collection CSVs.

  python scripts/pmc_summary.py out/run_counter_collection.csv [...]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    vals = defaultdict(list)
    for path in sys.argv[1:]:
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
                name = name.replace("void ", "")[:44]
                key = (name, int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0), r["Counter_Name"])
                vals[key].append(float(r["Counter_Value"]))
    print(f"{'kernel':44s} {'grid':>9s} {'counter':>22s} {'median':>14s}")
    for (n, g, c), v in sorted(vals.items()):
        print(f"{n:44s} {g:9d} {c:>22s} {statistics.median(v):14.1f}")


if __name__ == "__main__":
    main()
