#!/bin/bash
# Round-3 evidence pass (tool): the chip's random-gather ceiling (tools/ubench/chase), the C4
# bench line, its kernel trace, and per-kernel PMC passes (traffic, SQ issue/wait, L2 hit rate)
# of the check path.  Every GPU step has its own limit; a failure ends the run.
#   usage: tools/gpu_r03_probe.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r03a}
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
if [ -z "${SKIP_CHASE:-}" ]; then
  for L in 1 2 4 8; do
    for W in 1 4; do
      timeout -k 5 60 tools/ubench/chase 32768 8 $L 64 0 $W >> $O/chase.txt || { echo "chase failed"; exit 1; }
    done
  done
  timeout -k 5 60 tools/ubench/chase 32768 8 1 64 0 1 >> $O/chase.txt || exit 1
  cat $O/chase.txt
fi
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 10 > $O/kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-160
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 2 --warmup 0"
RX="fr_|resolve_kernel|fb_|blk_"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d $O/pmc$i -o pmc --output-format csv \
    -- python3 bench.py $ARGS > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/pmc$i.log; exit 1; }
done
python3 tools/pmc_split.py $O/pmc_split.json $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4
rm -rf $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/kt
