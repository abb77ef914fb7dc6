# the RCCL overlap probe with 1 vs 3 communicators (RCCL's own streams take hardware queues too)
mkdir -p gpurun_out/r4_pad
for c in 1 3; do
  for p in 0 6; do
    TZ_TEST_COMMS=$c TZ_PAD_STREAMS=$p OUT=r4_pad/ovlc_${c}_$p CASE=rccl_overlap T=150 bash scripts/rccl_loopback_diag.sh | grep RESULT \
      | sed "s/^RESULT {/{\"comms\": $c, \"pad\": $p, /" >> gpurun_out/r4_pad/rccl_comms.jsonl || exit $?
  done
done
cat gpurun_out/r4_pad/rccl_comms.jsonl | cut -c1-200
