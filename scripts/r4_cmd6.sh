# (b) user-level RCCL collectives between 2 loopback ranks; (a) the RCCL halo loopback test three
# times with every rank's log kept; then the storage-order table
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
mkdir -p gpurun_out/r4_faults
OUT=r4_faults/comm_ops CASE=comm_ops W=2 T=170 bash scripts/rccl_loopback_diag.sh > gpurun_out/r4_faults/comm_ops.txt 2>&1
rc=$?; echo "comm_ops rc=$rc"; grep -o '"runs": .*' gpurun_out/r4_faults/comm_ops.txt | cut -c1-300
if fatal $rc; then exit $rc; fi
for i in 1 2 3; do
  TZ_TEST_LOGDIR=gpurun_out/r4_faults/halo_rep$i timeout -k 10 175 python -u -m pytest tests/test_gpu_multirank.py -x -q \
    --timeout 170 --timeout-method thread -p no:cacheprovider -k "rccl_halo_across_ranks_loopback and 2" \
    > gpurun_out/r4_faults/halo_rep$i.log 2>&1
  rc=$?; echo "halo rep $i rc=$rc: $(tail -1 gpurun_out/r4_faults/halo_rep$i.log)"
  if fatal $rc; then exit $rc; fi
done
bash scripts/r4_layouts.sh
