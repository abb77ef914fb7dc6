#!/bin/bash
# The driver's 1-GPU bench with each of the 9 MCTS strategies (same 40-candidate budget, same
# seed): the best schedule each one finds, its timed value and the search wall-clock.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/strategies
mkdir -p "$OUT"
for s in FastMin Coverage Random AvgTime Unvisited AntiCorrelation NormalizedAntiCorrelation NormRootCorr BalanceHistogram; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --strategy $s > "$OUT/$s.json" 2> /dev/null
  rc=$?
  [ $rc -ne 0 ] && { echo "$s rc=$rc"; exit $rc; }
  python3 -c "import json;j=json.loads(open('$OUT/$s.json').read().strip().splitlines()[-1]);print('$s', round(j['value'],5), 'search_s', round(j['search_wall_s'],3), 'best_search', round(j['search_best_pct10_ms'],5), 'ops', j['schedule_ops'])"
done
exit 0
