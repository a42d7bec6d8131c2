#!/bin/bash
# fr_reduce A/B (tool): kernel-trace batch stats of bench.py's C4 batches, in-tree vs
# tools/ab/libketo_redser.so, and their pipelined / device-resident steps.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04red} && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for v in base redser base redser; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib
  timeout -k 10 300 python3 -u bench.py $A > $O/$v.log 2>&1 || { echo "$v failed"; exit 1; }
  tail -1 $O/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v value %.1fM step %.3f resident %.3f mism %s' % (d['value']/1e6, d['ms_per_step'], d['device_resident']['kernel_ms'], d['pipeline']['mismatches']))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 bench.py $A --steps 5 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; exit 1; }
  echo "  $(grep -E 'fr_reduce' $(find $O/kt_$v -name '*kernel_stats.csv') | cut -d, -f2-4)"
  rm -rf $O/kt_$v
done
