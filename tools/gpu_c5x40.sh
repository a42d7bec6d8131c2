#!/bin/bash
# config 5 at its configured size (tests/test_gpu_c5.py) after the partition tests of the same
# build; every GPU step bounded, the first failure ends the run.   usage: tools/gpu_c5x40.sh
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_partition.py \
  "tests/test_gpu_scale.py::test_c5_partitioned_one_rank" > gpurun_out/c5_part.log 2>&1 || { tail -30 gpurun_out/c5_part.log; exit 1; }
tail -3 gpurun_out/c5_part.log
free -g | head -2
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_c5.py > gpurun_out/c5x40.log 2>&1
rc=$?; grep -v "^$" gpurun_out/c5x40.log | tail -40; exit $rc
