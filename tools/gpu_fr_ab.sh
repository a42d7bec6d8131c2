#!/bin/bash
# frontier A/B: the in-tree library and every tools/ab/libketo_fr*.so on the Drive profiling batch
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for lib in djy-keto_amd/keto_mi355x/libketo_mi355x.so tools/ab/libketo_fr*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python3 -u tools/prof_check.py --workload drive --batches 0 --compare > gpurun_out/frab.log 2>&1 || { tail -5 gpurun_out/frab.log; exit 1; }
  grep -E "FRONTIER=1|identical" gpurun_out/frab.log
done
