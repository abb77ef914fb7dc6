# hipGraph branch concurrency against the number of streams the runtime owns
mkdir -p gpurun_out/r4_capture
for v in equal2:2 equal2:3 equal2:4 equal3:3 equal3:4 equal3:5 equal3:6 equal4:4 equal4:5 equal4:8; do
  TZ_OVERLAP_STREAMS=${v#*:} timeout -k 10 120 python -u scripts/child_graph_overlap.py ${v%:*} >> gpurun_out/r4_capture/nstreams.jsonl || exit $?
done
cat gpurun_out/r4_capture/nstreams.jsonl
