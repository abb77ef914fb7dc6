# capture root A/B on the hipGraph BASELINE configurations: c2g (SpMV DFS, every candidate a
# hipGraph) and c5 (SpMV + halo fused graph, MCTS, hipGraph candidates)
for r in none kernel; do
  TZ_GRAPH_ROOT=$r OUT=gpurun_out/r4_root/cfg_$r STEPS="c2g c5" bash scripts/baseline_configs.sh || exit $?
done
