#!/bin/bash
# The driver's 1-GPU bench with the round-1 batch sizing (close half the gap to the target per
# run) and the direct sizing, alternating: search wall-clock and the best schedule's time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sizing
for rep in $(seq 1 ${REPS:-3}); do
  for half in 1 0; do
    TZ_HALF_GAP_SIZING=$half timeout -k 10 240 python bench.py --steps 20 --warmup 5 \
      > gpurun_out/sizing/h${half}_$rep.json 2> /dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "half=$half rc=$rc"; exit $rc; }
    python3 -c "import json;j=json.loads(open('gpurun_out/sizing/h${half}_$rep.json').read().strip().splitlines()[-1]);print('half_gap=$half rep=$rep', round(j['value'],5), 'search_s', round(j['search_wall_s'],3), 'raced', j['mcts_raced'], 'best_search', round(j['search_best_pct10_ms'],5), 'rerank', [round(x,5) for x in j['rerank']['pct10_ms']])"
  done
done
exit 0
