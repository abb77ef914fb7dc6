#!/bin/bash
# Loopback (2 ranks on one GPU, receive buffers) A/B of the pack / unpack cache policies
# (TZ_NT_PACK: non-temporal grid loads in pack; TZ_NT_UNPACK: non-temporal ghost stores in
# unpack), alternating. Loopback shares one GPU's HBM between the ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nt_multi
export TMPDIR=/tmp TZ_IPC_GRID=0
for rep in 1 2; do
  for v in "1 0" "1 1" "0 1" "0 0"; do
    set -- $v
    TZ_NT_PACK=$1 TZ_NT_UNPACK=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29900 + rep * 10 + $1 * 2 + $2)) \
      bench.py --gpus 2 --steps 50 --warmup 10 --link-probe-iters 0 \
      > gpurun_out/nt_multi/p$1u$2_r$rep.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "p$1u$2 rc=$rc"; tail -3 gpurun_out/nt_multi/p$1u$2_r$rep.log; exit $rc; }
    python3 -c "import json;l=[x for x in open('gpurun_out/nt_multi/p$1u$2_r$rep.log') if x.startswith('{')][-1];j=json.loads(l);print('pack_nt=$1 unpack_nt=$2 rep=$rep', round(j['value'],4), j['schedule_transport'], j['verified_bad_cells'])"
  done
done
exit 0
