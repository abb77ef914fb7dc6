# A/B of the capture root (TZ_GRAPH_ROOT none / kernel / empty): branch probes, the RCCL overlap
# probe between 2 loopback ranks, and the driver's 1-GPU bench
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
out=gpurun_out/r4_root
mkdir -p $out
for r in none kernel empty; do
  for v in kernels equal3 equal4 host hostchain; do
    TZ_GRAPH_ROOT=$r timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"root\": \"$r\", /" >> $out/probes.jsonl
    rc=$?; if fatal $rc; then exit $rc; fi
  done
  TZ_GRAPH_ROOT=$r OUT=r4_root/ovl_$r CASE=rccl_overlap T=150 bash scripts/rccl_loopback_diag.sh | grep RESULT | sed "s/^RESULT {/{\"root\": \"$r\", /" >> $out/rccl.jsonl
  rc=$?; if fatal $rc; then exit $rc; fi
  TZ_GRAPH_ROOT=$r timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$r.json 2> $out/bench_$r.err
  rc=$?; echo "bench $r rc=$rc $(cut -c1-120 $out/bench_$r.json)"; if fatal $rc; then exit $rc; fi
done
cat $out/probes.jsonl
