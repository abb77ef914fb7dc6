#!/bin/bash
# Loopback A/B: the bench at N=2 and N=4 with and without copy-engine (SDMA) puts offered
# (TZ_IPC_COPY=0/1), receive-buffer mode. Loopback ranks share one GPU: HBM contention, not xGMI.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/put_ab2
export TMPDIR=/tmp TZ_IPC_GRID=0
for n in 2 4; do
  for copy in 0 1; do
    TZ_IPC_COPY=$copy timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29700 + n * 10 + copy)) bench.py --gpus $n --steps 50 \
      --warmup 10 > gpurun_out/put_ab2/n${n}_copy$copy.log 2>&1
    rc=$?
    echo "n=$n copy=$copy rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/put_ab2/n${n}_copy$copy.log; exit $rc; fi
  done
done
exit 0
