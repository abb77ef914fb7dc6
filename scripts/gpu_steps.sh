#!/bin/bash
# One GPU-box call as a list of steps, each with its own time limit:
#   scripts/gpu_steps.sh OUTDIR 'name|seconds|command' ...
# Each step's stdout+stderr goes to OUTDIR/name.log. A fault, abort or time limit (exit 124, 134,
# 137, 139) ends the call there; a plain failure (e.g. a failing test, exit 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  IFS='|' read -r name t cmd <<< "$step"
  echo "== $name ($(date +%T), limit ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"
  tail -c 800 "$OUT/$name.log" | tail -5
  case $rc in 124|134|137|139) echo "fatal rc in $name; stopping"; exit $rc;; esac
done
exit 0
