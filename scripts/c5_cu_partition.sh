set -u
mkdir -p gpurun_out/c5cu
for cfg in "2 --cu-partition" "4 --cu-partition" "2"; do
  set -- $cfg
  tag="s$1${2:+_cu}"
  timeout -k 10 200 python3 -m tenzing_amd search --workload fused --solver mcts --iters 150 --streams $cfg \
    --mode graph --graph-unroll 8 --neighbors 26 --order qxyz --bench-iters 20 --target-secs 0.004 \
    > gpurun_out/c5cu/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/c5cu/$tag.log | cut -c1-260
done
