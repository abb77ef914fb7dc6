#!/bin/bash
# Two settings of the driver's 1-GPU bench, alternating (A B A B ...): the timed value, the
# search wall-clock and the search's view of the best schedule.
#   A="--target-secs 0.002" B="--target-secs 0.001" REPS=3 bash scripts/bench_ab.sh
# (an entry may also start with ENV=value pairs, e.g. A="TZ_PREFLIGHT_S=5")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bench_ab
mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-3}); do
  for side in A B; do
    args=${!side}
    timeout -k 10 240 env ${args%%--*} python bench.py --steps 20 --warmup 5 \
      $( [[ "$args" == *--* ]] && echo "--${args#*--}" ) > "$OUT/${side}_$rep.json" 2> /dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "$side rc=$rc"; exit $rc; }
    python3 -c "import json;j=json.loads(open('$OUT/${side}_$rep.json').read().strip().splitlines()[-1]);print('$side rep=$rep', round(j['value'],5), 'search_s', round(j['search_wall_s'],3), 'raced', j['mcts_raced'], 'best_search', round(j['search_best_pct10_ms'],5), 'rerank', [round(x,5) for x in j['rerank']['pct10_ms']])"
  done
done
exit 0
