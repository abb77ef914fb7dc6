#!/bin/bash
# The driver's 1-GPU bench with and without racing, alternating: search wall-clock and the
# best schedule's time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/race
for rep in 1 2 3; do
  for r in 1.25 0; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --race-ratio $r > gpurun_out/race/r${r}_$rep.json 2> /dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "race=$r rc=$rc"; exit $rc; }
    python3 -c "import json;j=json.loads(open('gpurun_out/race/r${r}_$rep.json').read().strip().splitlines()[-1]);print('race=$r rep=$rep', round(j['value'],5), 'search_s', round(j['search_wall_s'],3), 'raced', j['mcts_raced'], 'best_search', round(j['search_best_pct10_ms'],5))"
  done
done
exit 0
