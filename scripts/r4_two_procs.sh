# two processes on the one GPU at once, each running a branch probe (the loopback setting of the
# RCCL probe, without RCCL): does sharing the GPU between processes cost graph concurrency?
mkdir -p gpurun_out/r4_pad
for v in equal2 equal3 hostchain; do
  for k in 1 2; do
    timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"procs\": 2, /" >> gpurun_out/r4_pad/two_procs.jsonl &
  done
  wait
  timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"procs\": 1, /" >> gpurun_out/r4_pad/two_procs.jsonl || exit $?
done
cat gpurun_out/r4_pad/two_procs.jsonl | cut -c1-160
