# spare-stream padding on the hipGraph BASELINE configurations: c2g (SpMV DFS, every candidate a
# hipGraph, 2 streams) and c5 (SpMV + halo fused graph, MCTS, hipGraph candidates, 4 streams)
for p in 0 6; do
  TZ_PAD_STREAMS=$p OUT=gpurun_out/r4_pad/cfg_$p STEPS="c2g c5" bash scripts/baseline_configs.sh || exit $?
done
