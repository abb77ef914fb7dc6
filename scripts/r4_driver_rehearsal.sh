#!/bin/bash
# Round 4. The driver's commands on one GPU: N=1 bench (+ a rocprofv3 kernel-stats pass), then the
# multi-rank command with N loopback ranks (all on this GPU; flow and robustness, not xGMI speed).
# N=8 is the driver's own case (its 8-GPU node) and is not run here by default.
# Every step has its own time limit; a crash, abort or time limit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUTD=${OUTD:-r4_rehearsal}
mkdir -p gpurun_out/$OUTD
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -z "${SKIP_N1:-}" ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${OUTD:-r4_rehearsal}/n1.json 2> gpurun_out/${OUTD:-r4_rehearsal}/n1.err
  rc=$?; echo "n=1 rc=$rc"; tail -c 600 gpurun_out/${OUTD:-r4_rehearsal}/n1.json; echo
  if fatal $rc; then exit $rc; fi
  if [ -n "${PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${OUTD:-r4_rehearsal}/prof -o run \
      -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${OUTD:-r4_rehearsal}/prof.log 2>&1
    rc=$?; echo "rocprof rc=$rc"
    if fatal $rc; then exit $rc; fi
    python3 scripts/trace_summary.py gpurun_out/${OUTD:-r4_rehearsal}/prof/run_kernel_trace.csv --last 300 \
      --timeline 80 --out gpurun_out/${OUTD:-r4_rehearsal}/prof/timeline.txt --delete > /dev/null || true
  fi
fi
port=29810
for n in ${NS:-2 4}; do
  port=$((port+1))
  timeout -k 10 ${NT:-560} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 20 --warmup 5 ${BENCH_ARGS:-} \
    > gpurun_out/${OUTD:-r4_rehearsal}/n$n.json 2> gpurun_out/${OUTD:-r4_rehearsal}/n$n.err
  rc=$?; echo "n=$n rc=$rc"; tail -c 800 gpurun_out/${OUTD:-r4_rehearsal}/n$n.json; echo
  if fatal $rc; then exit $rc; fi
done
# RCCL working between the loopback ranks (a host id per rank): RCCL is seeded and measured beside
# the IPC transports, its candidates compiled in whole-schedule capture
for n in ${RCCL_NS:-}; do
  port=$((port+1))
  TZ_RCCL_LOOPBACK=1 timeout -k 10 ${NT:-560} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 20 --warmup 5 --link-probe-rccl ${BENCH_ARGS:-} \
    > gpurun_out/$OUTD/rccl_n$n.json 2> gpurun_out/$OUTD/rccl_n$n.err
  rc=$?; echo "rccl n=$n rc=$rc"; tail -c 800 gpurun_out/$OUTD/rccl_n$n.json; echo
  if fatal $rc; then exit $rc; fi
done
exit 0
