#!/bin/bash
# Config 5 (C3 x10, one rank): L2 requests per kernel (TCC_HIT_sum + TCC_MISS_sum, one --pmc pass)
# over a short bench run, for where the batch's random accesses go.   usage: tools/gpu_c5_pmc.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5pmc} && rm -rf $O && mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmc -o pmc --output-format csv \
  -- python3 bench.py --workload c5 --scale 10 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1 \
  || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -1); cp "$f" $O/counters.csv; rm -rf $O/pmc
ls -la $O
