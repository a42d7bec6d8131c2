#!/bin/bash
# One GPU-box profiling pass of the default bench line: kernel-trace summary (per kernel and per
# 2^20 batch of the check path) and the HBM traffic passes.  Each GPU step has its own time limit
# and the first failure ends the run.   usage: tools/gpu_prof.sh r02 c4
set -eu
cd "$(dirname "$0")/.."
ROUND=${1:-r02}
WL=${2:-c4}
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/kt_$WL
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$WL -o kt --output-format csv \
  -- python3 bench.py --workload $WL --no-cpu-baseline --serve-clients 0 --latency-iters 0 > gpurun_out/kt_$WL.log 2>&1
grep "^{\"metric" gpurun_out/kt_$WL.log > gpurun_out/${ROUND}_kt_bench_$WL.json
KT=$(find gpurun_out/kt_$WL -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/kt_$WL -name "*kernel_stats.csv" | head -1)
cp "$ST" gpurun_out/${ROUND}_${WL}_kernel_stats.csv
python3 tools/kt_summary.py "$KT" gpurun_out/${ROUND}_${WL}_kernel_grid_stats.csv > /dev/null
python3 tools/kt_batches.py "$KT" --out gpurun_out/${ROUND}_${WL}_batch_stats.csv
tools/pmc_traffic.sh $ROUND $WL
cp gpurun_out/pmc_traffic_$WL/${ROUND}_traffic_$WL.json gpurun_out/
