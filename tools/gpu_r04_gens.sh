#!/bin/bash
# Async speculation depth learned on the device (tool): the frontier GPU tests, then the C5 x10
# one-rank line (every batch asynchronous) and the C4 line.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04gens} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
timeout -k 10 400 python3 -u bench.py --workload c5 --scale 10 --steps 20 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || { echo c5 failed; tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5x10 value %.1fM ms/step %.3f mism %s' % (d['value']/1e6, d['ms_per_step'], d['pipeline']['mismatches']))"
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe > $O/c4.log 2>&1 || { echo c4 failed; exit 1; }
tail -1 $O/c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 value %.1fM ms/step %.3f mism %s' % (d['value']/1e6, d['ms_per_step'], d['pipeline']['mismatches']))"
