# wide kernel puts: the new loopback tests, the bench tests that probe put_wide
mkdir -p gpurun_out/r4_wide
TZ_TEST_LOGDIR=gpurun_out/r4_wide/ranklogs timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider \
  -k "wide_puts or bench_two_ranks_loopback or ipc_halo_loopback" > gpurun_out/r4_wide/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r4_wide/pytest.log
exit $rc
