# graph-branch concurrency against the number of HIP hardware queues per process
mkdir -p gpurun_out/r4_capture
for q in 4 8 16; do
  for v in kernels kernel3 hostchain; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"hw_queues\": $q, /" >> gpurun_out/r4_capture/hwq.jsonl || exit $?
  done
done
cat gpurun_out/r4_capture/hwq.jsonl
