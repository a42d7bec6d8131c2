#!/bin/bash
# Same-box A/B of the two frontier engines on the C4 bench (device-resident and pipelined
# rates, kernel time): block (default) vs generation (KETO_FR_ENGINE=gen).  Each run bounded.
#   usage: tools/gpu_engine_ab.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r03ab}
O=gpurun_out/$TAG && rm -rf $O && mkdir -p $O
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 10 --steps 10"
for E in block gen block gen; do
  KETO_FR_ENGINE=$E KETO_FR_VERBOSE=${VERBOSE:-} timeout -k 10 300 python3 -u bench.py $ARGS > $O/bench_$E.log 2>&1 || { echo "bench $E failed"; tail -5 $O/bench_$E.log; exit 1; }
  tail -1 $O/bench_$E.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$E', 'value %.1fM' % (d['value']/1e6), 'resident %.1fM' % (d['device_resident']['checks_per_s']/1e6), 'kernel_ms %.3f' % d['device_resident']['kernel_ms'], 'goals', d.get('frontier',{}).get('goals_per_batch'))"
done
