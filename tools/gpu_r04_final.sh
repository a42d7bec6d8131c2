#!/bin/bash
# Round-4 measurements of the current build: sha-stamped traffic passes for C4 / C2 / C3
# (tools/pmc_traffic.sh), the C4 kernel-trace summary, then the bench lines (C4 default with its
# probes and CPU baseline, C5 x10 one rank, C2, C3) that report them.  Each GPU step bounded; a
# failure ends the run.   usage: tools/gpu_r04_final.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r04z} && rm -rf $O && mkdir -p $O
for w in c4 c2 c3; do
  bash tools/pmc_traffic.sh r04 $w > $O/pmc_$w.log 2>&1 || { echo "pmc $w failed"; tail -5 $O/pmc_$w.log; exit 1; }
  cp gpurun_out/pmc_traffic_$w/r04_traffic_$w.json $O/ && cp $O/r04_traffic_$w.json profiles/
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 10 --no-store-probe > $O/kt.log 2>&1 \
  || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
cp $(find $O/kt -name "*kernel_stats.csv" | head -1) $O/c4_kernel_stats.csv
python3 tools/kt_batches.py $(find $O/kt -name "*kernel_trace.csv" | head -1) > $O/c4_batch_stats.txt 2>&1 || true
tail -1 $O/kt.log > $O/kt_bench.json; rm -rf $O/kt
timeout -k 10 600 python3 -u bench.py > $O/bench_c4.log 2>&1 || { echo "c4 bench failed"; tail -8 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log > $O/bench_c4.json
timeout -k 10 400 python3 -u bench.py --workload c5 --scale 10 --steps 10 --warmup 2 > $O/bench_c5.log 2>&1 \
  || { echo "c5 bench failed"; tail -8 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log > $O/bench_c5_x10.json
for w in c2 c3; do
  timeout -k 10 400 python3 -u bench.py --workload $w --serve-clients 0 --no-store-probe > $O/bench_$w.log 2>&1 \
    || { echo "$w failed"; tail -5 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log > $O/bench_$w.json
done
for f in $O/*.json; do echo "$f"; cut -c1-300 $f; done
