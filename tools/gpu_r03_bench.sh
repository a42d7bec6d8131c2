#!/bin/bash
# The default bench line (C4, N=1) on the final build, with the round's traffic profile in
# profiles/ (tools/gpu_r03_final.sh made it for this library).   usage: tools/gpu_r03_bench.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03b} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_line.json
tail -1 $O/bench.log | cut -c1-1500
