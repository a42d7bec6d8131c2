#!/bin/bash
# quick pass: frontier GPU tests, C4 bench line (frontier stats, parity sample), C5 x10 one rank
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q_tests.log; if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/q_tests.log | head; exit $rc; fi
KETO_FR_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --serve-clients 0 --latency-iters 20 > gpurun_out/q_c4.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/q_c4.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('C4',d['value']/1e6,d['ms_per_step'],d['roofline']['kernel_ms'],d['frontier'],d['cpu_parity_sample'],d['p99_batch_latency_ms'])"
grep "^\[frontier\]" gpurun_out/q_c4.log | tail -1
KETO_PART_VERBOSE=1 KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 5 --warmup 1 > gpurun_out/q_c5.log 2>&1 || exit $?
grep '^{"metric' gpurun_out/q_c5.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('C5',d['value']/1e6,d['ms_per_step'],d['phases_ms_per_step'])"
grep "keto build" gpurun_out/q_c5.log | tail -5
