#!/bin/bash
# C5 phase breakdown (closure steps, build steps) + C4 bench line with the adaptive read-back
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
KETO_PART_VERBOSE=1 KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 3 --warmup 1 > gpurun_out/x_c5.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/x_c5.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('C5',d['value']/1e6,d['ms_per_step'],d['phases_ms_per_step'])"
grep -E "keto build|steps \(ms\)" gpurun_out/x_c5.log | tail -12
timeout -k 10 300 python3 -u bench.py --serve-clients 0 --latency-iters 20 --no-cpu-baseline > gpurun_out/x_c4.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/x_c4.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('C4',d['value']/1e6,d['ms_per_step'],d['roofline']['kernel_ms'],d['frontier'])"
