mkdir -p gpurun_out/r4_capture
TZ_LOG=debug timeout -k 10 200 python -u -X faulthandler scripts/r4_self_diag.py > gpurun_out/r4_capture/self_torchrt2.log 2>&1
rc=$?
echo "torch runtime rc=$rc"; tail -40 gpurun_out/r4_capture/self_torchrt2.log
exit $rc
