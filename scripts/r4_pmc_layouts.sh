#!/bin/bash
# HBM bytes of the 26-direction move in both storage orders (FETCH_SIZE, WRITE_SIZE: one counter
# group per rocprofv3 pass, each pass under a hard limit; a failed pass stops the script)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/r4_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for order in qxyz xyzq; do
  for group in FETCH_SIZE WRITE_SIZE; do
    TZ_PMC_ORDER=$order timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d "$OUT/${order}_$group" -o run \
      -- python3 "$ROOT/scripts/pmc_targets.py" --only-move 20 > "$OUT/${order}_$group.log" 2>&1
    rc=$?; echo "$order $group rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 "$ROOT/scripts/pmc_summary.py" $(find "$OUT" -path "*${order}_*" -name '*counter_collection.csv') > "$OUT/summary_$order.txt"
  cat "$OUT/summary_$order.txt"
done
find "$OUT" -name '*counter_collection.csv' -delete
