# host-side completion latency in the driver's N=1 command: HIP's default wait vs an active
# (spinning) wait before it blocks (CLR's ROC_ACTIVE_WAIT_TIMEOUT, microseconds)
mkdir -p gpurun_out/r4_sync_ab
for k in 1 2 3; do
  for w in default 100000; do
    if [ "$w" = default ]; then
      timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_sync_ab/${w}_$k.json 2> gpurun_out/r4_sync_ab/${w}_$k.err || exit $?
    else
      ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_sync_ab/${w}_$k.json 2> gpurun_out/r4_sync_ab/${w}_$k.err || exit $?
    fi
    python - "$w" "$k" <<'PY'
import json, sys
w, k = sys.argv[1:]
j = json.loads(open(f"gpurun_out/r4_sync_ab/{w}_{k}.json").read().strip().splitlines()[-1])
print(w, k, round(j["value"], 5), round(j["eager_ms_per_step"], 5))
PY
  done
done
