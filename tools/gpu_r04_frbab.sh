#!/bin/bash
# Block-engine A/B (tool): bench.py's C4 latency probe (64Ki batches, p99) and serving probe for the
# in-tree library and tools/ab variants, twice each.   usage: tools/gpu_r04_frbab.sh OUT name...
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/$1 && shift && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --no-store-probe --steps 5"
for r in 1 2; do for v in base "$@"; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py $A > $O/$v.$r.log 2>&1 \
    || { echo "$v failed"; tail -5 $O/$v.$r.log; exit 1; }
  tail -1 $O/$v.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['serving']; print('$v', 'p99 %.3f ms' % d['p99_batch_latency_ms'], 'serving %.2fM/s p99 %.2f ms' % (s['checks_per_s']/1e6, s['p99_request_ms']), 'value %.1fM' % (d['value']/1e6))"
done; done
