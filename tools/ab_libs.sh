#!/bin/bash
# A/B timing of alternative engine builds in tools/ab/ on C3 (and the current build); full
# output of each run in gpurun_out/ab_<name>.log.   usage: tools/ab_libs.sh [lib-glob]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in cur tools/ab/${1:-libketo_*.so}; do
  if [ "$lib" = cur ]; then unset KETO_MI355X_LIB_OVERRIDE KETO_MI355X_ALLOW_OVERRIDE; name=cur
  else export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; name=$(basename $lib .so); fi
  timeout -k 10 120 python3 tools/build_scale.py --scale ${SCALE:-1} --batches 4 > gpurun_out/ab_$name.log 2>&1
  rc=$?
  grep -E "batch 3|allowed" gpurun_out/ab_$name.log | sed "s/^/$name: /"
  if [ $rc -ne 0 ]; then echo "$name: rc=$rc"; tail -3 gpurun_out/ab_$name.log; exit 1; fi
done
