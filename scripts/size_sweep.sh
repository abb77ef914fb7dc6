#!/bin/bash
# Per-rank domain size sweep on one GPU: the headline bench (27-point halo, MCTS, hipGraph
# replay) at n^3 x 3 f64 per rank for growing n, up to a grid of ~207 GB (n = 2048) in one
# MI355X's 288 GB. Each size runs under its own time limit; a crash or timeout stops the sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/size_sweep
for n in ${SIZES:-256 512 1024 1536 2048}; do
  timeout -k 10 "${STEP_TIMEOUT:-240}" python bench.py --cells "$n" --steps 50 --warmup 10 \
    --mcts-iters "${MCTS_ITERS:-20}" > "gpurun_out/size_sweep/n$n.json" 2> "gpurun_out/size_sweep/n$n.err"
  rc=$?
  echo "n=$n rc=$rc $(tail -c 300 gpurun_out/size_sweep/n$n.json)"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/size_sweep/n$n.err"; exit $rc; fi
done
