# torch's bundled HIP 7.0.2 / RCCL 2.26.6 vs the system ROCm HIP 7.2 / RCCL 2.27.7 (TZ_NO_TORCH=1)
# on the driver's commands: N=1 twice each, loopback N=2, RCCL between loopback ranks at N=2
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
out=gpurun_out/r4_rt
mkdir -p $out
port=29650
for rep in 1 2; do
  for rt in torch system; do
    nt=""; [ $rt = system ] && nt=1
    TZ_NO_TORCH=$nt timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/n1_${rt}_$rep.json 2> $out/n1_${rt}_$rep.err
    rc=$?; echo "n1 $rt $rep rc=$rc"; if fatal $rc; then exit $rc; fi
  done
done
for rt in torch system; do
  nt=""; [ $rt = system ] && nt=1
  port=$((port+1))
  TZ_NO_TORCH=$nt timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 20 --warmup 5 > $out/n2_$rt.json 2> $out/n2_$rt.err
  rc=$?; echo "n2 $rt rc=$rc"; if fatal $rc; then exit $rc; fi
  port=$((port+1))
  TZ_NO_TORCH=$nt TZ_RCCL_LOOPBACK=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 20 --warmup 5 > $out/rccl_n2_$rt.json 2> $out/rccl_n2_$rt.err
  rc=$?; echo "rccl n2 $rt rc=$rc"; if fatal $rc; then exit $rc; fi
done
