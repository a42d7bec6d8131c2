#!/bin/bash
# regroup experiments: dispatch-key union cost with / without regrouping, then block sizes
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
export KETO_MI355X_ALLOW_OVERRIDE=tools
export KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_prof1.so
KETO_REGROUP=0 timeout -k 10 200 python3 tools/prof_states.py > gpurun_out/prof_off.log 2>&1 || exit $?
echo "== lane kernel"; cat gpurun_out/prof_off.log
timeout -k 10 200 python3 tools/prof_states.py > gpurun_out/prof_on.log 2>&1 || exit $?
echo "== regrouped"; cat gpurun_out/prof_on.log
for lib in cur tools/ab/libketo_rg256.so tools/ab/libketo_rg1024.so; do
  if [ $lib = cur ]; then unset KETO_MI355X_LIB_OVERRIDE; else export KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; fi
  timeout -k 10 200 python3 tools/prof_check.py --workload drive --count --batches 3 > gpurun_out/ab_rg.log 2>&1 || { tail -3 gpurun_out/ab_rg.log; exit 1; }
  echo "== $lib"; grep -E "tier 0|batch 2" gpurun_out/ab_rg.log
done
KETO_REGROUP=0 timeout -k 10 200 python3 tools/prof_check.py --workload drive --count --batches 3 > gpurun_out/ab_rg.log 2>&1 || exit 1
echo "== lane kernel"; grep -E "tier 0|batch 2" gpurun_out/ab_rg.log
