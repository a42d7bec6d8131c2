#!/bin/bash
# A/B of the block-regrouped interpreter: its parity tests, then the C4 bench line without and with it
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "regroup" > gpurun_out/rg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rg_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--workload ${WL:-c4} --steps 10 --warmup 2 --no-cpu-baseline --serve-clients 0 --latency-iters 0"
KETO_REGROUP=0 timeout -k 10 300 python3 -u bench.py $ARGS > gpurun_out/rg_off.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/rg_off.log').read().strip().splitlines()[-1]);print('off',d['value'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python3 -u bench.py $ARGS > gpurun_out/rg_on.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/rg_on.log').read().strip().splitlines()[-1]);print('on',d['value'],d['roofline']['kernel_ms'])"
