#!/bin/bash
# Round-4 capture diagnosis on one GPU: graph-branch overlap of two kernels (and of a host node
# beside them), whole-schedule vs child capture; then RCCL between two loopback ranks
# (TZ_RCCL_LOOPBACK=1): the overlap probe and the halo's RCCL transport eager + hipGraph over
# value generations, on torch's bundled runtime and (RTS) on the system ROCm runtime.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r4_capture}
mkdir -p "$out"
for cap in schedule child; do
  for v in kernels host; do
    TZ_GRAPH_CAPTURE=$cap timeout -k 10 120 python -u scripts/child_graph_overlap.py $v >> "$out/overlap.jsonl"
  done
done
cat "$out/overlap.jsonl"
for rt in ${RTS:-torch}; do
  nt=""; [ "$rt" = system ] && nt=1
  for k in 2 1; do
    TZ_NO_TORCH=$nt TZ_TEST_OVERLAP_KERNELS=$k OUT=${OUT:-r4_capture}/ovl_${rt}_k$k CASE=rccl_overlap T=${T:-150} \
      TZ_TEST_VERBOSE=1 bash scripts/rccl_loopback_diag.sh | grep RESULT
  done
  TZ_NO_TORCH=$nt OUT=${OUT:-r4_capture}/halo_$rt CASE=ipc_halo T=${T:-150} TZ_TEST_VERBOSE=1 \
    TZ_TEST_TRANSPORT=rccl TZ_TEST_SEEDS=2 bash scripts/rccl_loopback_diag.sh | grep -o '"transports": {[^}]*}\|"bad[123]": [0-9]*' | sort | uniq -c
done
