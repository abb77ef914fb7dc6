# graph-branch concurrency against HIP's graph execution stream count (DEBUG_HIP_FORCE_GRAPH_QUEUES)
mkdir -p gpurun_out/r4_capture
for q in default 1 2 4 8; do
  for v in kernels kernel3 kernel4 hostchain; do
    if [ $q = default ]; then
      timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"graph_queues\": \"$q\", /" >> gpurun_out/r4_capture/graphq.jsonl || exit $?
    else
      DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"graph_queues\": \"$q\", /" >> gpurun_out/r4_capture/graphq.jsonl || exit $?
    fi
  done
done
cat gpurun_out/r4_capture/graphq.jsonl
