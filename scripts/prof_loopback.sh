#!/bin/bash
# rocprofv3 kernel traces of the multi-rank bench with 2 ranks on this one GPU (loopback): one
# profiler per rank process (no launcher between the profiler and the program), each under its
# own time limit. Summaries of each rank's timed loop go to gpurun_out/prof_lb/r<rank>/.
# Loopback ranks share one GPU, so the puts, waits and unpacks show their kernel costs, not
# xGMI speed.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/prof_lb
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PORT=$((20000 + RANDOM % 20000))
pids=()
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r$r" -o run \
    -- python3 "$ROOT/bench.py" --gpus 2 --steps 60 --warmup 10 > "$OUT/r$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "ranks rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 0 1; do
  python3 "$ROOT/scripts/trace_summary.py" "$OUT/r$r/run_kernel_trace.csv" --last 400 --timeline 60 \
    --out "$OUT/r$r/timeline.txt" --delete > /dev/null
done
grep -h '^{"metric' "$OUT/r0.log" | tail -1 | cut -c1-300
head -14 "$OUT/r0/timeline.txt"
