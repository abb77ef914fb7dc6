#!/bin/bash
# Multi-rank BASELINE configurations in loopback: N ranks (processes) on the one GPU of a
# gpurun box, through the same torchrun launch the driver uses on an 8-GPU node. RCCL refuses
# several ranks on one device, so the workloads fall back (collectively) to IPC puts. Timings
# share one GPU between the ranks: they validate the flow, not xGMI speed.
# Results: gpurun_out/loopback_cfg/*.log (last line = JSON summary).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/loopback_cfg
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { # name nranks timeout args...
  local name=$1 n=$2 t=$3; shift 3
  timeout -k 10 "$t" python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) -m tenzing_amd search "$@" \
    --csv "$OUT/$name.csv" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-260)"
  if fatal $rc; then echo "fatal rc in $name; stopping"; exit $rc; fi
  return 0
}
S=${STEPS:-"spmv2 spmv4 fused2"}
[[ " $S " == *" spmv2 "* ]] && run spmv_mcts_n2 2 400 --workload spmv --solver mcts --iters 100 \
  --streams 2 --bench-iters 10 --target-secs 0.002
[[ " $S " == *" spmv4 "* ]] && run spmv_mcts_n4 4 400 --workload spmv --solver mcts --iters 100 \
  --streams 2 --bench-iters 10 --target-secs 0.002
[[ " $S " == *" fused2 "* ]] && run fused_mcts_graph_n2 2 600 --workload fused --solver mcts \
  --iters 100 --streams 4 --mode graph --graph-unroll 8 --neighbors 26 --order qxyz \
  --bench-iters 10 --target-secs 0.004
exit 0
