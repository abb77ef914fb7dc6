#!/bin/bash
# The driver's 1-GPU bench command at two graph unroll depths (iterations per hipGraph launch),
# alternating, so launch latency amortization can be compared at the driver's 20 timed steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/unroll
for rep in 1 2 3; do
  for u in 10 20; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --graph-unroll $u \
      > gpurun_out/unroll/u${u}_r$rep.json 2> /dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "u=$u rc=$rc"; exit $rc; }
    python3 -c "import json;j=json.loads(open('gpurun_out/unroll/u${u}_r$rep.json').read().strip().splitlines()[-1]);print('u=$u rep=$rep', round(j['value'],5))"
  done
done
exit 0
