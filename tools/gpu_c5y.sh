#!/bin/bash
# partition GPU tests (C5 at size included) + the C5 bench line with step breakdown
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_partition.py tests/test_gpu_scale.py -k "partition or c5" -x -q --timeout 450 --timeout-method thread > gpurun_out/y_tests.log 2>&1
rc=$?; tail -2 gpurun_out/y_tests.log; if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/y_tests.log | head; exit $rc; fi
KETO_PART_VERBOSE=1 KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 5 --warmup 1 > gpurun_out/y_c5.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/y_c5.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('C5',d['value']/1e6,d['ms_per_step'],d['phases_ms_per_step'])"
grep -E "steps \(ms\)" gpurun_out/y_c5.log | tail -2
