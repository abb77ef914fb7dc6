# N equal 200 us kernels, eager and hipGraph, against GPU_MAX_HW_QUEUES (HIP's default is 4)
mkdir -p gpurun_out/r4_capture
for q in 8 16; do
  for e in 0 1; do
    for v in equal3 equal4 equal6 equal8; do
      GPU_MAX_HW_QUEUES=$q TZ_OVERLAP_EAGER=$e timeout -k 10 120 python -u scripts/child_graph_overlap.py $v \
        | sed "s/^{/{\"hw_queues\": $q, /" >> gpurun_out/r4_capture/equal_hwq.jsonl || exit $?
    done
  done
done
cat gpurun_out/r4_capture/equal_hwq.jsonl
