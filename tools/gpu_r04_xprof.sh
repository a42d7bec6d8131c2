#!/bin/bash
# expand_wave on C4 (tool): kernel trace of bench.py's expand probe and PMC passes restricted to
# the Expand kernels (SQ waves / waits / instruction mix, L2 requests, HBM bytes).  Each pass its
# own run, bounded; a failure ends the run.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04xp} && rm -rf $O && mkdir -p $O
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 2 --warmup 0 --no-store-probe"
RX="expand_"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py $A > $O/kt.log 2>&1 || { echo kt failed; exit 1; }
cp $(find $O/kt -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d $O/pmc$i -o pmc --output-format csv -- python3 bench.py $A > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name "*counter_collection.csv" | head -1); cp $f $O/pmc$i.csv
done
rm -rf $O/kt $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/pmc5
grep -i expand $O/kernel_stats.csv | cut -d, -f1-4
