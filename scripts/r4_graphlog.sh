# HIP's own account of how it runs a graph launch (AMD_LOG_LEVEL=4, filtered to its graph lines)
mkdir -p gpurun_out/r4_capture/graphlog
for v in equal2 equal3 equal4; do
  AMD_LOG_LEVEL=4 timeout -k 10 120 python -u scripts/child_graph_overlap.py $v 2>&1 \
    | grep -E "hipGraph\]|GraphExec|max streams|parallel streams|^\{" | sort | uniq -c | sort -rn | head -40 \
    > gpurun_out/r4_capture/graphlog/$v.txt
  rc=$?; echo "$v rc=$rc"; head -20 gpurun_out/r4_capture/graphlog/$v.txt
done
