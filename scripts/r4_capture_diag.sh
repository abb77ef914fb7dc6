#!/bin/bash
# Round-4 capture diagnosis on one GPU: flat-vs-child overlap of two kernels, then RCCL between
# two loopback ranks (TZ_RCCL_LOOPBACK=1) in whole-schedule capture: the overlap probe and the
# halo's RCCL transport eager + hipGraph over value generations. Every step has its own limit;
# the first failure ends the script.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r4_capture}
mkdir -p "$out"
for cap in schedule child; do
  TZ_GRAPH_CAPTURE=$cap timeout -k 10 120 python -u scripts/child_graph_overlap.py >> "$out/overlap.jsonl"
done
cat "$out/overlap.jsonl"
for cap in ${CAPS:-schedule}; do
  TZ_GRAPH_CAPTURE=$cap OUT=${OUT:-r4_capture}/ovl_$cap CASE=rccl_overlap T=${T:-150} TZ_TEST_VERBOSE=1 bash scripts/rccl_loopback_diag.sh
  TZ_GRAPH_CAPTURE=$cap OUT=${OUT:-r4_capture}/halo_$cap CASE=ipc_halo T=${T:-150} TZ_TEST_VERBOSE=1 \
    TZ_TEST_TRANSPORT=rccl TZ_TEST_SEEDS=2 TZ_TEST_NO_MCTS=${NO_MCTS:-} bash scripts/rccl_loopback_diag.sh
done
