#!/bin/bash
# Round-end GPU pass on the final build: the -m gpu suite, the default bench line, its kernel-trace
# summary (probes off: every check-path launch is a 2^20 batch's) and the PMC traffic passes
# (profiles/<round>_traffic_c4.json is stamped with this library's sha256).  Every GPU step has
# its own limit; a timeout, abort or crash ends the run.   usage: tools/gpu_final.sh r02
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
ROUND=${1:-r02}
timeout -k 10 780 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
rm -rf gpurun_out/kt_final
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_final -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 > gpurun_out/kt_final.log 2>&1 || { echo "kernel trace failed"; exit 1; }
f=$(find gpurun_out/kt_final -name "*kernel_trace.csv" | head -1)
python3 tools/kt_summary.py "$f" gpurun_out/${ROUND}_c4_kernel_grid_stats.csv > /dev/null
python3 tools/kt_batches.py "$f" --out gpurun_out/${ROUND}_c4_batch_stats.csv | tail -6
cp $(find gpurun_out/kt_final -name "*kernel_stats.csv" | head -1) gpurun_out/${ROUND}_c4_kernel_stats.csv
bash tools/pmc_traffic.sh $ROUND c4 > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc.log; exit 1; }
tail -1 gpurun_out/pmc.log
