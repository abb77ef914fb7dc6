mkdir -p gpurun_out/r4_cli
TZ_TEST_LOGDIR=gpurun_out/r4_cli/ranklogs timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider \
  -k "native_cli or save_best or bench_save" > gpurun_out/r4_cli/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -10 gpurun_out/r4_cli/pytest.log; exit $rc
