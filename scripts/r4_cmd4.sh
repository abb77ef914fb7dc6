# capture check: RCCL self-exchange diag, the runtime GPU tests, then the RCCL loopback probes
mkdir -p gpurun_out/r4_capture
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
TZ_LOG=debug timeout -k 10 200 python -u -X faulthandler scripts/r4_self_diag.py > gpurun_out/r4_capture/self_torchrt3.log 2>&1
rc=$?; echo "self diag rc=$rc"; grep -v "Debug" gpurun_out/r4_capture/self_torchrt3.log | tail -12
if fatal $rc; then exit $rc; fi
timeout -k 10 480 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_capture/pytest_rt.log 2>&1
rc=$?; echo "pytest runtime rc=$rc"; tail -5 gpurun_out/r4_capture/pytest_rt.log
if fatal $rc; then exit $rc; fi
bash scripts/r4_capture_diag.sh
