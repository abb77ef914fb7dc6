# N 200 us kernels forked from one root vs N independent roots, hipGraph and eager
mkdir -p gpurun_out/r4_capture
for e in 0 1; do
  for v in equal3 fork3 fork4 fork6; do
    TZ_OVERLAP_EAGER=$e timeout -k 10 120 python -u scripts/child_graph_overlap.py $v >> gpurun_out/r4_capture/fork.jsonl || exit $?
  done
done
cat gpurun_out/r4_capture/fork.jsonl
