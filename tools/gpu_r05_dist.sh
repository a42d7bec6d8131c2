#!/bin/bash
# round 5: the distributed frontier's GPU tests (two gloo ranks sharing the GPU) + the single-GPU
# frontier suites it shares its kernels with, then a short C4 bench (refactor check)
set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py \
    tests/test_gpu_spine.py tests/test_gpu_frontier.py > gpurun_out/r05a/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r05a/bench.log 2>&1
