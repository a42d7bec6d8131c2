#!/bin/bash
# tools/gpu_final.sh, then the config-5 bench line (C3 x10, one rank) of the same build.
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_final.sh ${1:-r02} || exit $?
timeout -k 10 400 python3 -u bench.py --workload c5 --scale 10 --steps 10 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || { echo "c5 bench failed"; tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-200
