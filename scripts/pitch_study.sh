#!/bin/bash
# The reference layout's move time on this box: XYZQ with x = 0 at the row
# start, row pitch 528 doubles (the reference's 4224 B) and 528 + 8 / 16 / 32, timed against its
# shape-matched roof (scripts/roof_probe.py), then the move's HBM traffic and L2 behaviour under
# rocprofv3 counters, one pass per counter group, at pitch 528 and 544. Run it on two boxes
# (two gpurun calls) and compare: a counter that moves with the time names the cause.
#
#   TAG=boxA bash scripts/pitch_study.sh        -> gpurun_out/r6_pitch/boxA/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O="gpurun_out/r6_pitch/${TAG:-box}"
mkdir -p "$O"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

# the box: GPU model, partition modes (they set how addresses interleave over HBM channels)
{ rocm-smi --showproductname --showmemorypartition --showcomputepartition 2>&1 || true; } > "$O/box.txt"

timeout -k 10 300 python3 scripts/roof_probe.py --iters 20 \
  --layouts xyzq:-1:0,xyzq:-1:8,xyzq:-1:16,xyzq:-1:32,xyzq:16:0,qxyz:16:0 > "$O/roof.jsonl" 2> "$O/roof.err"
rc=$?; echo "roof_probe rc=$rc"
if fatal $rc; then exit $rc; fi

i=0
for pad in 0 16; do
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    d="$O/pmc_p${pad}_$i"
    TZ_PMC_ORDER=xyzq TZ_PMC_ALIGN=-1 TZ_PMC_PITCH_PAD=$pad timeout -s KILL 90 \
      rocprofv3 --pmc $ctr --output-format csv -d "$d" -o run -- python3 scripts/pmc_targets.py --only-move 20 \
      > "$d.log" 2>&1
    rc=$?; echo "pmc pad=$pad [$ctr] rc=$rc"
    if fatal $rc; then exit $rc; fi
    f=$(find "$d" -name '*counter_collection.csv' | head -n 1)
    if [ -n "$f" ]; then
      python3 scripts/pmc_summary.py "$f" | grep -E 'kernel|box_move' > "$d.txt"
      rm -rf "$d"
    fi
  done
done
exit 0
