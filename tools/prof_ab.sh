#!/bin/bash
# A/B hardware-counter passes of tools/prof_check.py for the current build and tools/ab/libketo_v1.so.
# Each rocprofv3 --pmc pass runs alone under its own hard timeout (MI355X_MICROARCH.md rocprofv3 notes).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "list failed"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for lib in cur v1; do
  if [ $lib = v1 ]; then export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_v1.so; else unset KETO_MI355X_LIB_OVERRIDE; fi
  timeout -k 10 120 python3 tools/prof_check.py --batches 3 > $OUT/time_$lib.txt 2>&1 || { echo "timing $lib failed"; exit 1; }
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/${lib}_p$i -o pmc --output-format csv -- python3 tools/prof_check.py --batches 2 > $OUT/${lib}_p$i.log 2>&1 || { echo "pmc pass $i $lib failed rc=$?"; tail -5 $OUT/${lib}_p$i.log; }
  done
done
echo done
