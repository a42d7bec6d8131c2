#!/bin/bash
# C3/C4/C5 at-size parity (frontier path) + the default C4 bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_SCALE:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/scale_tests.log 2>&1 || { tail -40 gpurun_out/scale_tests.log; exit 1; }
  tail -2 gpurun_out/scale_tests.log
fi
timeout -k 10 500 python3 -u bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || { tail -30 gpurun_out/bench_c4.log; exit 1; }
tail -3 gpurun_out/bench_c4.log
