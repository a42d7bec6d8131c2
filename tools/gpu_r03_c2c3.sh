#!/bin/bash
# The C2 and C3 lines of the final build (bench.py --workload c2 / c3; probes off).
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03c23} && rm -rf $O && mkdir -p $O
for w in c2 c3; do
  timeout -k 10 400 python3 -u bench.py --workload $w --serve-clients 0 --no-store-probe > $O/bench_$w.log 2>&1 \
    || { echo "$w failed"; tail -5 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log > $O/bench_$w.json; cut -c1-300 $O/bench_$w.json
done
