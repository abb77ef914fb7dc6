set -u
mkdir -p gpurun_out/lb
export TMPDIR=/tmp
for n in ${NS:-2 4}; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) bench.py --gpus $n --steps 50 --warmup 10 > gpurun_out/lb/bench_n$n.log 2>&1
  rc=$?; echo "n=$n rc=$rc"; tail -1 gpurun_out/lb/bench_n$n.log | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
exit 0
