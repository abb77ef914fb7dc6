#!/bin/bash
# BASELINE configs 2 (SpMV, DFS over every schedule) with racing: the same exhaustive search,
# clearly slow candidates cut short after 2 measurements. SETTLE_ONLY=1: with settling too
# (a candidate whose first 4 measurements agree within 3 % is done).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/race_configs
mkdir -p "$OUT"
run() { # name args...
  local name=$1; shift
  timeout -k 10 600 python3 -m tenzing_amd search "$@" --csv "$OUT/$name.csv" > "$OUT/$name.log" 2>&1
  local rc=$?
  [ $rc -ne 0 ] && { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json;j=[json.loads(l) for l in open('$OUT/$name.log') if l.startswith('{') and 'best_pct10_ms' in l][-1];print('$name', j['candidates'], round(j['best_pct10_ms']*1e3,2), 'us', round(j['search_wall_s'],2), 's')"
}
if [ -n "${SETTLE_ONLY:-}" ]; then
  run c2g_settle --workload spmv --solver dfs --max-seqs 15000 --streams 2 --mode graph --graph-unroll 8 --bench-iters 20 --target-secs 0.002 --race-ratio 1.25 --settle-ratio 0.03
  run c2_settle --workload spmv --solver dfs --max-seqs 15000 --streams 2 --bench-iters 20 --target-secs 0.002 --race-ratio 1.25 --settle-ratio 0.03
  exit 0
fi
run c2_race --workload spmv --solver dfs --max-seqs 15000 --streams 2 --bench-iters 20 --target-secs 0.002 --race-ratio 1.25
run c2g_race --workload spmv --solver dfs --max-seqs 15000 --streams 2 --mode graph --graph-unroll 8 --bench-iters 20 --target-secs 0.002 --race-ratio 1.25
exit 0
