#!/bin/bash
# round 5: config 5 on the distributed frontier -- the C5 test's flow at x${KETO_C5_SCALE:-10} (8 gloo ranks
# sharing the GPU), then the bench's 8-rank rehearsal line at the same scale
set -o pipefail
OUT=gpurun_out/${R05_TAG:-r05c}
mkdir -p $OUT
export KETO_C5_SCALE=${KETO_C5_SCALE:-10}
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 980 --timeout-method thread tests/test_gpu_c5.py > $OUT/c5test.log 2>&1 || exit $?
cp gpurun_out/c5x40_phases.json $OUT/c5_phases_x${KETO_C5_SCALE}.json
KETO_BENCH_BACKEND=gloo KETO_POOL_CAP_MB=1 KETO_SCRATCH_CAP_MB=1 KETO_PART_TRIM=1 timeout -k 10 900 \
    python -u bench.py --workload c5 --scale $KETO_C5_SCALE --gpus 8 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c5bench.log 2>&1
