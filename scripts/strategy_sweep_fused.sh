#!/bin/bash
# Each of the 9 MCTS strategies on the largest 1-GPU decision tree (BASELINE config 5: SpMV +
# 27-point halo in one graph, 4 streams, hipGraph candidates), same budget and seed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/strategies_fused
mkdir -p "$OUT"
for s in FastMin Coverage Random AvgTime Unvisited AntiCorrelation NormalizedAntiCorrelation NormRootCorr BalanceHistogram; do
  timeout -k 10 300 python -m tenzing_amd search --workload fused --solver mcts --iters ${ITERS:-60} \
    --streams 4 --mode graph --graph-unroll 8 --neighbors 26 --order qxyz --bench-iters 10 \
    --target-secs 0.002 --race-ratio 1.25 --strategy $s --csv "$OUT/$s.csv" > "$OUT/$s.json" 2> /dev/null
  rc=$?
  [ $rc -ne 0 ] && { echo "$s rc=$rc"; exit $rc; }
  python3 -c "import json;j=json.loads(open('$OUT/$s.json').read().strip().splitlines()[-1]);print('$s', 'best_us', round(j['best_pct10_ms']*1e3,2), 'search_s', round(j['search_wall_s'],2), 'candidates', j['candidates'])"
done
exit 0
