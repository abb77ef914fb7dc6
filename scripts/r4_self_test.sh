mkdir -p gpurun_out/r4_self_overlap
TZ_TEST_LOGDIR=gpurun_out/r4_self_overlap/ranklogs timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider \
  -k "overlaps_kernels" > gpurun_out/r4_self_overlap/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r4_self_overlap/pytest.log; exit $rc
