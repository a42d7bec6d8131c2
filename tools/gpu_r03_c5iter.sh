#!/bin/bash
# One GPU call while iterating on the config-5 path: the -m gpu suite (config 5 at x40 aside),
# then tools/gpu_c5_prof.sh (the C3 x10 one-rank line with phase times, and its kernel trace).
#   usage: tools/gpu_r03_c5iter.sh tag
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03i} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_c5.py::test_c5_x40_eight_ranks_matches_oracle > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
bash tools/gpu_c5_prof.sh ${1:-r03i}_c5 10
