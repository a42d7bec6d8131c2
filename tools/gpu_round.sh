#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, its kernel-trace summary and the
# HBM traffic passes.  Every GPU step has its own time limit; the first failure ends the run.
# The kernel trace runs the bench without the latency and serving probes, so that every check
# launch it averages is a 2^20-query batch, the launch the bench line times.
#   usage: tools/gpu_round.sh r01 c4 [skip-tests]
set -eu
cd "$(dirname "$0")/.."
ROUND=${1:-r01}
WL=${2:-c4}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${3:-}" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 400 python3 -u bench.py --workload $WL > gpurun_out/bench_$WL.log 2>&1
tail -1 gpurun_out/bench_$WL.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$WL -o kt --output-format csv \
  -- python3 bench.py --workload $WL --no-cpu-baseline --serve-clients 0 --latency-iters 0 > gpurun_out/kt_$WL.log 2>&1
tail -1 gpurun_out/kt_$WL.log
tools/pmc_traffic.sh $ROUND $WL
