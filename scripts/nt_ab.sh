#!/bin/bash
# The driver's 1-GPU bench command with the move kernel's cache policy alternating between the
# default (plain loads, non-temporal ghost stores) and round 1's (non-temporal loads, plain stores).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nt_ab
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export TZ_NT_MOVE_LOAD=1 TZ_NT_MOVE_STORE=0; else unset TZ_NT_MOVE_LOAD TZ_NT_MOVE_STORE; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/nt_ab/${v}_r$rep.json 2> /dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "$v rc=$rc"; exit $rc; }
    python3 -c "import json;j=json.loads(open('gpurun_out/nt_ab/${v}_r$rep.json').read().strip().splitlines()[-1]);print('$v rep=$rep', round(j['value'],5), j['verified_bad_cells'])"
  done
done
exit 0
