#!/bin/bash
# Hardware counters of the headline kernel at steady state: the 26-direction move launched back
# to back (scripts/pmc_targets.py --only-move). One counter group per rocprofv3 pass, each pass
# under its own hard time limit; a failed pass stops the script. Summary:
# gpurun_out/pmc_move/summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/pmc_move
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$ROOT/scripts/pmc_targets.py" --only-move 20 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 "$ROOT/scripts/pmc_summary.py" $(find "$OUT" -name '*counter_collection.csv') > "$OUT/summary.txt"
find "$OUT" -name '*counter_collection.csv' -delete
cat "$OUT/summary.txt"
