#!/bin/bash
# Config 5 (C3 x10, one rank): pipelined vs one-after-another batches (KETO_PART_SEQUENTIAL), each
# twice, alternating, on fresh batches.   usage: tools/gpu_c5_seq_ab.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03sq} && rm -rf $O && mkdir -p $O
ARGS="--workload c5 --scale 10 --steps 10 --warmup 2 --no-cpu-baseline"
for i in 1 2; do
  for mode in pipe seq; do
    if [ $mode = seq ]; then export KETO_PART_SEQUENTIAL=1; else unset KETO_PART_SEQUENTIAL; fi
    timeout -k 10 300 python3 -u bench.py $ARGS > $O/$mode$i.log 2>&1 || { echo "$mode failed"; tail -5 $O/$mode$i.log; exit 1; }
    tail -1 $O/$mode$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', $i, 'ms/step %.2f' % d['ms_per_step'], 'value %.1fM' % (d['value']/1e6))"
  done
done
