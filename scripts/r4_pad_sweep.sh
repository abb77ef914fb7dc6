# spare-stream padding sweep: branch probes and the 2-rank RCCL probe
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
out=gpurun_out/r4_pad
mkdir -p $out
for p in 5 6 8; do
  for v in equal3 hostchain; do
    TZ_PAD_STREAMS=$p timeout -k 10 120 python -u scripts/child_graph_overlap.py $v | sed "s/^{/{\"pad\": $p, /" >> $out/probes.jsonl
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
for p in 0 4 5 6 8; do
  TZ_PAD_STREAMS=$p OUT=r4_pad/ovl_$p CASE=rccl_overlap T=150 bash scripts/rccl_loopback_diag.sh | grep RESULT | sed "s/^RESULT {/{\"pad\": $p, /" >> $out/rccl.jsonl
  rc=$?; if fatal $rc; then exit $rc; fi
done
