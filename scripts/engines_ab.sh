#!/bin/bash
# Loopback A/B of the copy engines per copy-engine put (TZ_COPY_ENGINES), 2 and 4 ranks on one
# GPU, receive-buffer mode: the bench's one-transfer probe and the exchange time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/engines
export TMPDIR=/tmp TZ_IPC_GRID=0
for n in 2 4; do
  for e in 1 2 4; do
    TZ_COPY_ENGINES=$e timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29800 + n * 10 + e)) bench.py --gpus $n --steps 50 \
      --warmup 10 > gpurun_out/engines/n${n}_e$e.log 2>&1
    rc=$?
    echo "n=$n engines=$e rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/engines/n${n}_e$e.log; exit $rc; fi
  done
done
exit 0
