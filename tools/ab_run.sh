#!/bin/bash
# A/B (tool): tier-0 kernel time and per-tier work of the current build and every tools/ab lib
# on the prof_check Drive workload.   usage: tools/ab_run.sh [drive|c2]
cd "$(dirname "$0")/.."
shopt -s nullglob
mkdir -p gpurun_out
for lib in cur tools/ab/libketo_*.so; do
  if [ $lib = cur ]; then unset KETO_MI355X_LIB_OVERRIDE; else export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; fi
  timeout -k 10 200 python3 tools/prof_check.py --workload ${1:-drive} --count --batches 3 > gpurun_out/ab_run.log 2>&1 || { tail -3 gpurun_out/ab_run.log; exit 1; }
  echo "== $lib"; grep -E "tier 0|tier 1|batch 2" gpurun_out/ab_run.log
done
