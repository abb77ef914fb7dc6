#!/bin/bash
# Each of the 9 MCTS strategies, same budget and seed: the best schedule each one finds.
#   WORKLOAD=halo  (default) the driver's 1-GPU bench: timed value and search wall-clock
#   WORKLOAD=fused BASELINE config 5 (SpMV + 27-point halo, 4 streams, hipGraph candidates),
#                  ITERS MCTS iterations (default 60)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=${WORKLOAD:-halo}
OUT=gpurun_out/strategies_$W
mkdir -p "$OUT"
for s in FastMin Coverage Random AvgTime Unvisited AntiCorrelation NormalizedAntiCorrelation NormRootCorr BalanceHistogram; do
  if [ "$W" = fused ]; then
    timeout -k 10 300 python -m tenzing_amd search --workload fused --solver mcts --iters ${ITERS:-60} \
      --streams 4 --mode graph --graph-unroll 8 --neighbors 26 --order qxyz --bench-iters 10 \
      --target-secs 0.002 --race-ratio 1.25 --strategy $s --csv "$OUT/$s.csv" > "$OUT/$s.json" 2> /dev/null
  else
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --subrecords off --strategy $s \
      > "$OUT/$s.json" 2> /dev/null
  fi
  rc=$?
  [ $rc -ne 0 ] && { echo "$s rc=$rc"; exit $rc; }
  python3 - "$OUT/$s.json" "$s" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if "best_pct10_ms" in j:
    print(sys.argv[2], "best_us", round(j["best_pct10_ms"] * 1e3, 2), "search_s", round(j["search_wall_s"], 2),
          "candidates", j["candidates"])
else:
    print(sys.argv[2], round(j["value"], 5), "search_s", round(j["search_wall_s"], 3),
          "best_search", round(j["search_best_pct10_ms"], 5), "ops", j["schedule_ops"])
PY
done
exit 0
