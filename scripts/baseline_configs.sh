#!/bin/bash
# The BASELINE.json configurations that fit one GPU box, each under its own time limit.
# Results (one JSON summary per config + search CSVs) go to gpurun_out/baseline/.
#   c1: no-op op graph, DFS full enumeration, host executor (no GPU)
#   c2: CSR SpMV (m=150000, nnz=10m), 1 GPU, DFS exhaustive over 2 HIP streams (c2g: every
#       candidate compiled to a hipGraph)
#   c4: 3-D 27-point halo, 512^3 x 3q, ghost 3, MCTS, 4 streams (bench.py; 1 rank here)
#   c5: SpMV + halo fused graph, MCTS with hipGraph-compiled candidates (1 rank here)
# The 2- and 8-rank variants (c3, c4 @ 8, c5 @ 8) need a multi-GPU node: bench.py under
# torchrun (the driver's scaling run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -c 400 "$OUT/$name.log" | tail -1 | cut -c1-300)"
  if fatal $rc; then echo "fatal rc in $name; stopping"; exit $rc; fi
  return 0
}
S=${STEPS:-"c1 c2 c2g c4 c5"}
[[ " $S " == *" c1 "* ]] && run c1_noop_dfs 300 python3 -m tenzing_amd search --workload noop \
  --noop-width 3 --solver dfs --streams 2 --bench-iters 20 --target-secs 0.002 \
  --csv "$OUT/c1_noop_dfs.csv"
[[ " $S " == *" c2 "* ]] && run c2_spmv_dfs 600 python3 -m tenzing_amd search --workload spmv \
  --solver dfs --max-seqs 15000 --streams 2 --bench-iters 20 --target-secs 0.002 \
  --csv "$OUT/c2_spmv_dfs.csv"
[[ " $S " == *" c2g "* ]] && run c2g_spmv_dfs_graph 600 python3 -m tenzing_amd search --workload spmv \
  --solver dfs --max-seqs 15000 --streams 2 --mode graph --graph-unroll 8 --bench-iters 20 --target-secs 0.002 \
  --csv "$OUT/c2g_spmv_dfs_graph.csv"
[[ " $S " == *" c4 "* ]] && run c4_halo_mcts 600 python3 bench.py --steps 500 --warmup 50 \
  --csv "$OUT/c4_halo_mcts.csv"
[[ " $S " == *" c5 "* ]] && run c5_fused_mcts 900 python3 -m tenzing_amd search --workload fused \
  --solver mcts --iters 150 --streams 4 --mode graph --graph-unroll 8 --neighbors 26 --order qxyz \
  --bench-iters 20 --target-secs 0.004 --csv "$OUT/c5_fused_mcts.csv"
exit 0
