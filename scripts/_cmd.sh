set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_runtime.py -x -q -p no:cacheprovider > gpurun_out/pyt.log 2>&1
rc=$?; tail -5 gpurun_out/pyt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_direct.log 2>&1 || exit $?
tail -1 gpurun_out/bench_direct.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --transport copy > gpurun_out/bench_copy.log 2>&1 || exit $?
tail -1 gpurun_out/bench_copy.log
STEPS="prof" PROF_ARGS="--steps 60 --warmup 10" bash scripts/gpu_round.sh
