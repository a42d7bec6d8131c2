#!/bin/bash
# regroup A/B: parity (forced regroup), then tier-0 kernel times of the lane kernel, the current
# regrouped build and tools/ab variants on the Drive workload
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "regroup" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
KETO_REGROUP=0 timeout -k 10 200 python3 tools/prof_check.py --workload drive --count --batches 3 > gpurun_out/ab_rg.log 2>&1 || exit 1
echo "== lane kernel"; grep -E "tier 0|batch 2" gpurun_out/ab_rg.log
export KETO_MI355X_ALLOW_OVERRIDE=tools
for lib in cur tools/ab/libketo_*.so; do
  if [ $lib = cur ]; then unset KETO_MI355X_LIB_OVERRIDE; else export KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; fi
  timeout -k 10 200 python3 tools/prof_check.py --workload drive --count --batches 3 > gpurun_out/ab_rg.log 2>&1 || { tail -3 gpurun_out/ab_rg.log; exit 1; }
  echo "== $lib"; grep -E "tier 0|batch 2" gpurun_out/ab_rg.log
done
