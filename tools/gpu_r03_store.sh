#!/bin/bash
# Incremental snapshots on the GPU: the store tests (patched vs full builds), then the C4 bench
# line with its store probe.  Every GPU step bounded; the first failure ends the run.
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03st} && rm -rf $O && mkdir -p $O
KETO_PATCH_VERBOSE=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_store.py > $O/store_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|patch\]" $O/store_tests.log | tail -30
[ $rc -ne 0 ] && { tail -30 $O/store_tests.log; exit $rc; }
KETO_PATCH_VERBOSE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
grep -v "^{" $O/bench.log | tail -12
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','ms_per_step','device_resident','incremental_snapshot','expand']: print(k, json.dumps(d.get(k))[:700])"
