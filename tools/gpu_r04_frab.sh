#!/bin/bash
# fr_expand compile-variant A/B (tool): bench.py's C4 line (probes off) for the in-tree library and
# the tools/ab/libketo_<name>.so variants given, twice each, one box.   usage: tools/gpu_r04_frab.sh OUT name...
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/$1 && shift && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for r in 1 2; do for v in base "$@"; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py $A > $O/$v.$r.log 2>&1 \
    || { echo "$v failed"; tail -5 $O/$v.$r.log; exit 1; }
  tail -1 $O/$v.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; f=d['frontier']; print('$v', 'value %.1fM' % (d['value']/1e6), 'step %.3f' % d['ms_per_step'], 'resident kernel %.3f' % d['device_resident']['kernel_ms'], 'goals %.1fM' % (f['goals_per_batch']/1e6), 'mism', p['mismatches'])"
done; done
