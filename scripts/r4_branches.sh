# graph-branch concurrency: 2, 3, 4 independent kernel branches, hipGraph vs eager
mkdir -p gpurun_out/r4_capture
for e in 0 1; do
  for v in kernels kernel3 kernel4; do
    TZ_OVERLAP_EAGER=$e timeout -k 10 120 python -u scripts/child_graph_overlap.py $v >> gpurun_out/r4_capture/branches.jsonl || exit $?
  done
done
cat gpurun_out/r4_capture/branches.jsonl
