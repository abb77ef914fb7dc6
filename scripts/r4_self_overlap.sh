# the RCCL overlap probe in ONE process: a 1-rank communicator, send/recv to itself, beside two
# ~200 us kernels (no second process on the GPU, no network proxy)
mkdir -p gpurun_out/r4_self_overlap
for c in 1 3; do
  TZ_TEST_COMMS=$c W=1 OUT=r4_self_overlap/c$c CASE=rccl_overlap T=120 bash scripts/rccl_loopback_diag.sh | grep RESULT \
    | sed "s/^RESULT {/{\"comms\": $c, /" >> gpurun_out/r4_self_overlap/self.jsonl || exit $?
done
cut -c1-400 gpurun_out/r4_self_overlap/self.jsonl
