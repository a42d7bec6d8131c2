#!/bin/bash
# quick GPU pass: selected tests, then a C5 bench with the builder's phase timing
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partition.py -x -q --timeout 300 --timeout-method thread -k "relation_error or partition or golden" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; grep "keto build" gpurun_out/bench_c5.log | tail -22; tail -1 gpurun_out/bench_c5.log; exit $rc
