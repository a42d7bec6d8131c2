#!/bin/bash
# Config 5 on the GPU: a one-rank C3 x10 bench line with the builder's phase times (where a
# closure batch's time goes), then config 5 at its size (tests/test_gpu_c5.py: C3 x40, 8 gloo
# ranks sharing the GPU).  Each step bounded; the first failure ends the run.
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5} && rm -rf $O && mkdir -p $O
KETO_BUILD_VERBOSE=1 timeout -k 10 400 python3 -u bench.py --workload c5 --scale 10 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5x10.log 2>&1 \
  || { echo "c5 x10 bench failed"; tail -8 $O/c5x10.log; exit 1; }
grep "keto build" $O/c5x10.log | tail -30
grep '^{' $O/c5x10.log | cut -c1-900
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 980 --timeout-method thread tests/test_gpu_c5.py > $O/c5x40.log 2>&1
rc=$?; grep -E "^\[c5|passed|failed|Error|assert" $O/c5x40.log | tail -60
exit $rc
