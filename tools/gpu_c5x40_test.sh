#!/bin/bash
# Config 5 at its configured size (tests/test_gpu_c5.py): 8 gloo ranks sharing the box's GPU,
# C3 x40 (4.22B tuples) partitioned by object.  One bounded step.
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5} && rm -rf $O && mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 980 --timeout-method thread tests/test_gpu_c5.py > $O/c5x40.log 2>&1
rc=$?; grep -E "^\[c5|passed|failed|Error|assert" $O/c5x40.log | tail -80
exit $rc
