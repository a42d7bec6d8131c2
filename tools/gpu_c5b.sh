#!/bin/bash
# C5 + frontier-default pass: partition and frontier GPU tests, then the C5 (x10, one rank) and C2
# bench lines with phase logs.  Each GPU step has its own limit; a crash ends the run.
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partition.py tests/test_gpu_frontier.py tests/test_gpu_scale.py -k "partition or c5 or frontier or union or routed" -x -q --timeout 500 --timeout-method thread > gpurun_out/c5b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c5b_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/c5b_tests.log | head -20; exit $rc; fi
KETO_PART_VERBOSE=1 KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 5 --warmup 1 > gpurun_out/c5b_bench.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/c5b_bench.log | cut -c1-200
grep -E "keto build|level [0-4]:" gpurun_out/c5b_bench.log | tail -10
timeout -k 10 300 python3 -u bench.py --workload c2 --serve-clients 0 > gpurun_out/c2b_bench.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/c2b_bench.log | cut -c1-300
