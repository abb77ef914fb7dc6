# A/B of the spare-stream padding (TZ_PAD_STREAMS 0 vs 4): branch probes, the RCCL probe between
# 2 loopback ranks (3 schedule streams), the 1-GPU bench
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
out=gpurun_out/r4_pad
mkdir -p $out
for p in 0 4; do
  for v in kernels equal3 equal4 host hostchain; do
    TZ_PAD_STREAMS=$p timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"pad\": $p, /" >> $out/probes.jsonl
    rc=$?; if fatal $rc; then exit $rc; fi
  done
  TZ_PAD_STREAMS=$p OUT=r4_pad/ovl_$p CASE=rccl_overlap T=150 bash scripts/rccl_loopback_diag.sh | grep RESULT | sed "s/^RESULT {/{\"pad\": $p, /" >> $out/rccl.jsonl
  rc=$?; if fatal $rc; then exit $rc; fi
  TZ_PAD_STREAMS=$p timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$p.json 2> $out/bench_$p.err
  rc=$?; echo "bench $p rc=$rc"; if fatal $rc; then exit $rc; fi
done
