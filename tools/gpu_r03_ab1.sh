#!/bin/bash
# store tests, then a C4 A/B of the in-tree build against tools/ab variants, then the default bench
# line (with its incremental-snapshot probe).  Every GPU step bounded; a failure ends the run.
#   usage: tools/gpu_r03_ab1.sh tag variant...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG && rm -rf $O && mkdir -p $O
KETO_PATCH_VERBOSE=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_store.py > $O/store_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert |patch\]" $O/store_tests.log | tail -20
[ $rc -ne 0 ] && { tail -30 $O/store_tests.log; exit $rc; }
bash tools/gpu_c4_ab.sh "$@" || exit 1
KETO_PATCH_VERBOSE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
grep -v "^{" $O/bench.log | tail -12
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','ms_per_step','device_resident','incremental_snapshot','expand','frontier']: print(k, json.dumps(d.get(k))[:700])"
