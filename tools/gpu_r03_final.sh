#!/bin/bash
# Round-3 evidence for the final build: the C4 kernel trace (rocprofv3 --kernel-trace --stats),
# the check path's HBM traffic (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.sh), per-kernel
# SQ / TCC counters (tools/pmc_split.py), then the default bench line that reports them.  Each
# GPU step has its own limit; a failure ends the run.   usage: tools/gpu_r03_final.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03f} && rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 10 --no-store-probe > $O/kt.log 2>&1 \
  || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
python3 tools/kt_batches.py $(find $O/kt -name "*kernel_trace.csv" | head -1) > $O/batch_stats.txt 2>&1 || true
head -14 $O/kernel_stats.csv | cut -c1-200
bash tools/pmc_traffic.sh r03 c4 || { echo "pmc traffic failed"; exit 1; }
cp gpurun_out/pmc_traffic_c4/r03_traffic_c4.json $O/
cat $O/r03_traffic_c4.json
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 2 --warmup 0 --no-store-probe"
RX="fr_|resolve_kernel"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d $O/pmc$i -o pmc --output-format csv \
    -- python3 bench.py $ARGS > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/pmc$i.log; exit 1; }
done
python3 tools/pmc_split.py $O/pmc_split.json $O/pmc3 $O/pmc4 $O/pmc1 $O/pmc2 || echo "split failed (not fatal)"
rm -rf $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 $O/kt
cp $O/r03_traffic_c4.json profiles/ 2>/dev/null  # (so the bench line below reports it)
[ -n "${NO_BENCH:-}" ] && exit 0  # (the bench line in a call of its own: tools/gpu_r03_bench.sh)
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
