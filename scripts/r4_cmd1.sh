mkdir -p gpurun_out/r4_capture
timeout -k 10 480 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_capture/pytest_rt.log 2>&1
rc=$?
tail -5 gpurun_out/r4_capture/pytest_rt.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
bash scripts/r4_capture_diag.sh
