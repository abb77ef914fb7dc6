#!/bin/bash
# Confirmation of the default box-move block order: GPU suite and smoke at the default, then
# 5 alternating headline bench pairs, round-robin (TZ_XCD_REMAP=0) vs the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xcdc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4 5; do
  for r in 0 default; do
    if [ $r = default ]; then env -u TZ_XCD_REMAP timeout -k 10 200 python bench.py --steps 300 --warmup 30 > $OUT/bench_${r}_$i.log 2>&1
    else TZ_XCD_REMAP=0 timeout -k 10 200 python bench.py --steps 300 --warmup 30 > $OUT/bench_${r}_$i.log 2>&1; fi
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $OUT/bench_${r}_$i.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$r',$i,round(d['value']*1e3,2),'us bad',d['verified_bad_cells'])" $OUT/bench_${r}_$i.log
  done
done
