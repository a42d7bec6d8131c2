#!/bin/bash
# One GPU call, several measurements (the pool is congested): the -m gpu suite (config 5 at x40
# aside), the C4 patch probe, a C4 A/B of the tools/ab variants named, a PC-sampling pass of
# fr_expand, the default bench line.  Each step bounded; the first failure ends the run.
#   usage: tools/gpu_r03_multi.sh tag variant...
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_c5.py::test_c5_x40_eight_ranks_matches_oracle > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
KETO_PATCH_VERBOSE=1 timeout -k 10 400 python3 -u tools/patch_probe.py 10 > $O/patch_probe.log 2>&1 || { echo "patch probe failed"; tail -5 $O/patch_probe.log; exit 1; }
grep -E "keto patch|patch_ms" $O/patch_probe.log | cut -c1-400
bash tools/gpu_c4_ab.sh "$@" || exit 1
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ['value','ms_per_step','device_resident','pipeline','incremental_snapshot','cpu_baseline','schedule_sensitivity','roofline']: print(k, json.dumps(d.get(k))[:500])"
exit 0
