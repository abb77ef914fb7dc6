# RCCL self-exchange under whole-schedule capture: native backtrace of the crash (pytest -s keeps
# stderr), torch's runtime first, then (only if that did not crash) the system ROCm runtime
mkdir -p gpurun_out/r4_capture
TZ_LOG=debug timeout -k 10 200 python -u -X faulthandler -m pytest tests/test_gpu_runtime.py -x -q -s \
  --timeout 120 --timeout-method thread -k "rccl_self" > gpurun_out/r4_capture/self_torchrt.log 2>&1
rc=$?
echo "torch runtime rc=$rc"; tail -40 gpurun_out/r4_capture/self_torchrt.log
case $rc in 0|1) ;; *) exit $rc;; esac
TZ_NO_TORCH=1 TZ_LOG=debug timeout -k 10 200 python -u -X faulthandler scripts/r4_self_diag.py > gpurun_out/r4_capture/self_sysrt.log 2>&1
rc=$?
echo "system runtime rc=$rc"; tail -40 gpurun_out/r4_capture/self_sysrt.log
exit $rc
