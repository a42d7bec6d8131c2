#!/bin/bash
# One GPU call: the -m gpu suite (config 5 at x40 aside), the default bench line, then config 5
# at its configured size (tests/test_gpu_c5.py).  Each step bounded; a failed step ends the run.
#   usage: tools/gpu_r03_verify.sh tag
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03v} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_c5.py::test_c5_x40_eight_ranks_matches_oracle > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','ms_per_step','device_resident','pipeline','p99_batch_latency_ms','serving','expand','incremental_snapshot','roofline']: print(k, json.dumps(d.get(k))[:600])"
timeout -k 10 1000 python3 -u -m pytest -x -v -s --timeout 980 --timeout-method thread tests/test_gpu_c5.py > $O/c5x40.log 2>&1
rc=$?; grep -E "^\[c5|passed|failed|Error|assert" $O/c5x40.log | tail -40
exit $rc
