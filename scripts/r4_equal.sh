# how many independent branches does a hipGraph launch run at once? N equal 200 us kernels
mkdir -p gpurun_out/r4_capture
for e in 0 1; do
  for v in equal2 equal3 equal4 equal6 equal8; do
    TZ_OVERLAP_EAGER=$e timeout -k 10 120 python -u scripts/child_graph_overlap.py $v >> gpurun_out/r4_capture/equal.jsonl || exit $?
  done
done
cat gpurun_out/r4_capture/equal.jsonl
