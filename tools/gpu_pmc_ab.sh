#!/bin/bash
# SQ instruction / cycle counters of the lane-resident and the block-regrouped interpreter
# (Drive workload, one 2^20 batch), one rocprofv3 --pmc pass each
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for mode in 0 1; do
  rm -rf gpurun_out/pmc_rg$mode
  KETO_REGROUP=$mode timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_rg$mode -o pmc --output-format csv -- python3 tools/prof_check.py --workload drive --batches 1 > gpurun_out/pmc_rg$mode.log 2>&1 || exit $?
  echo "== KETO_REGROUP=$mode"; python3 tools/pmc_sum.py gpurun_out/pmc_rg$mode
done
