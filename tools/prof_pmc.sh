#!/bin/bash
# Hardware-counter passes of tools/prof_check.py (current build), one rocprofv3 --pmc run per
# pass under its own hard timeout (MI355X_MICROARCH.md rocprofv3 notes).  $1 = workload (c2|drive)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
WL=${1:-c2}
OUT=gpurun_out/pmc_$WL
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
P4="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o pmc --output-format csv -- python3 tools/prof_check.py --batches 1 --workload $WL > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
