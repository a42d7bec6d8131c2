#!/bin/bash
# round 5: the distributed frontier's GPU tests (two gloo ranks sharing the GPU) + the single-GPU
# frontier suites it shares its kernels with, the x40 partition footprint, then a short C4 bench
set -o pipefail
OUT=gpurun_out/${R05_TAG:-r05b}
mkdir -p $OUT
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    "tests/test_gpu_partition.py::test_two_rank_partitioned_matches_oracle" > $OUT/t0.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py \
    tests/test_gpu_spine.py tests/test_gpu_frontier.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/dist_mem_probe.py --scale 40 --world 8 --rank 0 > $OUT/mem.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1
