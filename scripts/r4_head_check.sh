# HEAD check: full GPU suite + smoke, then the driver's commands (N=1 + kernel stats; loopback
# N=2 / 4; RCCL between loopback ranks at N=2), then the RCCL overlap probe
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/r4_suite.sh; rc=$?
if fatal $rc; then exit $rc; fi
OUTD=r4_head PROF=1 NS="2 4" RCCL_NS="2" bash scripts/r4_driver_rehearsal.sh; rc=$?
if fatal $rc; then exit $rc; fi
OUT=r4_head/ovl CASE=rccl_overlap T=150 bash scripts/rccl_loopback_diag.sh | grep RESULT > gpurun_out/r4_head/rccl_overlap.txt
