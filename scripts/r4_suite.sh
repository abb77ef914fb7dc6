# the full GPU suite, verbose (a hang names its test), then smoke
mkdir -p gpurun_out/r4_suite
TZ_TEST_LOGDIR=gpurun_out/r4_suite/ranklogs timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4_suite/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -15 gpurun_out/r4_suite/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_suite/smoke.txt 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/r4_suite/smoke.txt
exit $rc
