#!/bin/bash
# Expand A/B (tool): bench.py's C4 expand probe for the in-tree library and tools/ab variants,
# each under the KETO_XW_BPC values given.   usage: tools/gpu_r04_xab.sh OUT "lib:bpc ..."
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/$1 && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 2 --no-store-probe"
for v in $2; do
  name=${v%%:*}; bpc=${v##*:}
  if [ $name = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$name.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib KETO_XW_BPC=$bpc timeout -k 10 300 python3 -u bench.py $A > $O/$name.$bpc.log 2>&1 \
    || { echo "$v failed"; tail -5 $O/$name.$bpc.log; exit 1; }
  tail -1 $O/$name.$bpc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['expand']; print('$v', 'api %.3f'%x['ms_per_batch'], 'walk %.3f'%x['traversal_kernel_ms'], 'err', x['errors'], 'nodes', x['nodes_per_batch'])"
done
