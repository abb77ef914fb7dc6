#!/bin/bash
# BASELINE honesty table: the driver's 1-GPU bench command in both storage orders (QXYZ, ours;
# XYZQ, the reference driver's, tenzing-mcts/examples/halo_run_strategy.hpp:42-49) with 26 and 6
# neighbours, then rocprofv3 kernel stats of the XYZQ runs. Every step bounded; a crash stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4_layouts
mkdir -p "$out"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for order in qxyz xyzq; do
  for nb in 26 6; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --order $order --neighbors $nb \
      > "$out/${order}_${nb}.json" 2> "$out/${order}_${nb}.err"
    rc=$?; echo "$order $nb rc=$rc: $(cut -c1-160 "$out/${order}_${nb}.json")"
    if fatal $rc; then exit $rc; fi
  done
done
for nb in 26 6; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_xyzq_$nb" -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --order xyzq --neighbors $nb --mcts-iters 12 \
    > "$out/prof_xyzq_$nb.log" 2>&1
  rc=$?; echo "rocprof xyzq $nb rc=$rc"
  if fatal $rc; then exit $rc; fi
  python3 scripts/trace_summary.py "$out/prof_xyzq_$nb/run_kernel_trace.csv" --last 300 --timeline 60 \
    --out "$out/prof_xyzq_$nb/timeline.txt" --delete > /dev/null
done
exit 0
