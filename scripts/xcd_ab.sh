#!/bin/bash
# A/B of an XCD-aware block order of the box-move kernel (TZ_XCD_REMAP=MODE): GPU suite with the
# remap on, then the headline bench alternating off/on in separate processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xcd; mkdir -p $OUT
export TMPDIR=/tmp
TZ_XCD_REMAP=${MODE:-2} timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_remap.log 2>&1
rc=$?; echo "pytest remap rc=$rc"; tail -2 $OUT/pytest_remap.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for r in 0 ${MODE:-2}; do
    TZ_XCD_REMAP=$r timeout -k 10 200 python bench.py --steps 300 --warmup 30 > $OUT/bench_r${r}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $OUT/bench_r${r}_$i.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('remap',$r,'run',$i,round(d['value']*1e3,2),'us bad',d['verified_bad_cells'])" $OUT/bench_r${r}_$i.log
  done
done
