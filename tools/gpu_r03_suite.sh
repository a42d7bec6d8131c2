#!/bin/bash
# Round-3 GPU pass: the -m gpu suite without config 5 at x40, then config 5 at x40
# (tests/test_gpu_c5.py), then the default bench line and the block engine's (A/B).
# Every GPU step bounded; the first failure ends the run.
#   usage: tools/gpu_r03_suite.sh [tag] [skip-c5]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r03s}
O=gpurun_out/$TAG && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_c5.py::test_c5_x40_eight_ranks_matches_oracle > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log
[ $rc -ne 0 ] && { grep -E "Error|error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-900
KETO_FR_ENGINE=block timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 10 --steps 10 > $O/bench_block.log 2>&1 || { echo "bench block failed"; tail -5 $O/bench_block.log; exit 1; }
tail -1 $O/bench_block.log | cut -c1-400
if [ -z "${2:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_c5.py > $O/c5x40.log 2>&1
  rc=$?; grep -E "^\[c5|passed|failed|Error|assert|^[0-9] \{" $O/c5x40.log | tail -60
  [ $rc -ne 0 ] && { tail -30 $O/c5x40.log; exit $rc; }
  KETO_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --workload c5 --gpus 8 --steps 3 --warmup 1 > $O/bench_c5.log 2>&1 \
    || { echo "c5 bench failed"; tail -8 $O/bench_c5.log; exit 1; }
  grep '^{' $O/bench_c5.log | cut -c1-1500
fi
exit 0
