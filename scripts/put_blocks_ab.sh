#!/bin/bash
# Loopback A/B of the put kernels' block cap (TZ_PUT_MAX_BLOCKS): 2 ranks on one GPU, buffers
# mode, the bench's per-link probe and exchange time. Loopback puts go through the IPC mapping of
# the same GPU's memory, so this shows the cap's effect on that path only, not xGMI.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/put_ab
export TMPDIR=/tmp TZ_IPC_GRID=0
for cap in ${CAPS:-64 4096 16 256}; do
  TZ_PUT_MAX_BLOCKS=$cap timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + cap % 1000)) bench.py --gpus 2 --steps 50 --warmup 10 \
    --mcts-iters 60 > gpurun_out/put_ab/cap$cap.log 2>&1
  rc=$?; echo "cap=$cap rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/put_ab/cap$cap.log; exit $rc; }
done
exit 0
