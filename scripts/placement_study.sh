#!/bin/bash
# The reference layout's move on several grids of one process (scripts/placement_probe.py):
# per-grid move times, then per-grid counters, one rocprofv3 pass per counter group, for the
# groups this box's rocprofv3 lists.
#   TAG=x bash scripts/placement_study.sh      -> gpurun_out/r6_pitch/place_x/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O="gpurun_out/r6_pitch/place_${TAG:-box}"
mkdir -p "$O"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
{ rocm-smi --showproductname 2>&1 | grep -E "GUID" || true; } > "$O/box.txt"
timeout -s KILL 60 rocprofv3 --list-avail > "$O/avail.txt" 2>&1
echo "list-avail rc=$?"
G=${GRIDS:-6}
timeout -k 10 300 python3 scripts/placement_probe.py --grids $G --spacer-mb ${SPACER:-0} > "$O/times.jsonl" 2> "$O/times.err"
rc=$?; echo "times rc=$rc"; cat "$O/times.jsonl" | cut -c1-200
if fatal $rc; then exit $rc; fi
i=0
# GRBM_GUI_ACTIVE in every pass: the dispatch's own duration in GPU cycles (dispatches are
# serialized under counter collection), beside the counters of that same dispatch
for grp in "GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
           "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum" \
           "GRBM_GUI_ACTIVE TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum" \
           "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "GRBM_GUI_ACTIVE TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"; do
  ok=1
  for c in $grp; do grep -q "${c%_sum}" "$O/avail.txt" || ok=0; done
  if [ $ok -eq 0 ]; then echo "skip [$grp]: not listed"; continue; fi
  i=$((i + 1))
  d="$O/pmc_$i"
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$d" -o run -- \
    python3 scripts/placement_probe.py --grids $G --spacer-mb ${SPACER:-0} --iters 2 > "$d.log" 2>&1
  rc=$?; echo "pmc [$grp] rc=$rc"
  if fatal $rc; then exit $rc; fi
  f=$(find "$d" -name '*counter_collection.csv' | head -n 1)
  if [ -n "$f" ]; then
    python3 scripts/placement_probe.py --dispatches "$f" --grids $G > "$d.jsonl"
    grep -h move_us "$d.log" | cut -c1-160 > "$d.times" || true
    rm -rf "$d"
  fi
done
gzip -9 "$O/avail.txt"
exit 0
