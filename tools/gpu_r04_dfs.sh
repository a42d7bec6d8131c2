#!/bin/bash
# Async DFS fallback A/B (tool): bench.py C2 and C4 lines for the in-tree library (empty-list early
# exit, one routed query per wave) and tools/ab/libketo_dfsold.so (before).  Probes off.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04dfs} && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for w in c2 c4; do for v in base dfsold base dfsold; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --workload $w $A > $O/$w.$v.log 2>&1 \
    || { echo "$w $v failed"; tail -5 $O/$w.$v.log; exit 1; }
  tail -1 $O/$w.$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; print('$w $v', 'value %.1fM' % (d['value']/1e6), 'ms/step %.3f' % d['ms_per_step'], 'pipe kernel %.3f' % p['kernel_ms_per_batch'][0], 'resident %.3f' % d['device_resident']['ms_per_step'], 'mism', p['mismatches'])"
done; done
