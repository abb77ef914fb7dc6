#!/bin/bash
# One GPU-box session: GPU tests, then a short bench, then (optionally) a rocprofv3 profile.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script (exit codes
# 124/137 timeout, 134 abort, 139 segfault). Plain test failures (exit 1) do not stop later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests bench}"

fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

if [[ " $STEPS " == *" tests "* ]]; then
  timeout -k 10 "${TEST_TIMEOUT:-900}" python -m pytest tests -m gpu -x -q -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest -m gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  if fatal $rc; then echo "fatal rc in tests; stopping"; exit $rc; fi
fi

if [[ " $STEPS " == *" bench "* ]]; then
  timeout -k 10 "${BENCH_TIMEOUT:-600}" python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  if fatal $rc; then echo "fatal rc in bench; stopping"; exit $rc; fi
fi

if [[ " $STEPS " == *" prof "* ]]; then
  timeout -k 10 "${PROF_TIMEOUT:-600}" rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof -o run -- python3 bench.py ${PROF_ARGS:---mcts-iters 6 --steps 20 --warmup 5} \
    > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  if fatal $rc; then exit $rc; fi
  # the full trace is far too large to travel back: keep a summary of the timed loop
  python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv --last "${PROF_LAST:-300}" \
    --timeline "${PROF_TIMELINE:-80}" --out gpurun_out/prof/timeline.txt --delete > /dev/null
fi
exit 0
