mkdir -p gpurun_out/r4_links
TZ_TEST_LOGDIR=gpurun_out/r4_links/ranklogs timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider \
  -k "links_cli or bench_two_ranks_loopback" > gpurun_out/r4_links/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r4_links/pytest.log; exit $rc
