#!/bin/bash
# value pipeline over 1 / 2 / 3 engine streams (tool): bench.py's C4 line, probes off
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
OUT=$1; mkdir -p $OUT
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for k in 1 2 3 1; do
  timeout -k 10 300 python3 -u bench.py $ARGS --engine-streams $k > $OUT/s$k.log 2>&1 || { echo "$k failed"; tail -5 $OUT/s$k.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value %.1fM' % (d['value']/1e6), 'ms/step %.3f' % d['ms_per_step'], 'mism', d['pipeline'].get('mismatches'))" $OUT/s$k.log $k
done
