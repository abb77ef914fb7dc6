mkdir -p gpurun_out/r4_capture
for v in kernels kernel3 host hostchain chainhost; do
  timeout -k 10 120 python -u scripts/child_graph_overlap.py $v >> gpurun_out/r4_capture/overlap2.jsonl || exit $?
done
cat gpurun_out/r4_capture/overlap2.jsonl
