#!/bin/bash
# End-of-round check of this tree on a fresh box, as the driver runs it: smoke(), the -m gpu
# suite (config 5 at its configured size included).   usage: tools/gpu_r03_endcheck.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03e} && rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -8 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 980 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && grep -E "Error|assert|FAIL" $O/tests.log | head -20
exit $rc
