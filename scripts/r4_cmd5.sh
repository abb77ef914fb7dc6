# full GPU suite + smoke, then the user-level RCCL collectives between 2 loopback ranks (the
# round-3 diag_ops hang), then the storage-order table (bench + rocprof)
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/r4_suite.sh; rc=$?
if fatal $rc; then exit $rc; fi
OUT=r4_comm_ops CASE=comm_ops W=2 T=200 TZ_TEST_VERBOSE=1 bash scripts/rccl_loopback_diag.sh > gpurun_out/r4_comm_ops.txt 2>&1
rc=$?; echo "comm_ops rc=$rc"; grep -o '"runs": .*' gpurun_out/r4_comm_ops.txt | cut -c1-400
if fatal $rc; then exit $rc; fi
bash scripts/r4_layouts.sh
