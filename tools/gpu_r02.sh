#!/bin/bash
# One GPU-box pass for round 2: the whole -m gpu suite (configured-size C3/C4/C5 included), then
# the default bench line.  Each GPU step has its own time limit; a timeout, abort or crash of a
# step ends the run (plain test failures still let the bench run).
#   usage: tools/gpu_r02.sh [tests|bench|both] [extra bench args...]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
WHAT=${1:-both}
shift || true
if [ "$WHAT" != "bench" ]; then
  timeout -k 10 780 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -4 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
fi
if [ "$WHAT" != "tests" ]; then
  timeout -k 10 400 python3 -u bench.py "$@" > gpurun_out/bench.log 2>&1
  rc=$?
  tail -1 gpurun_out/bench.log
  exit $rc
fi
