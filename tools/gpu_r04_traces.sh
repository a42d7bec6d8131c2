#!/bin/bash
# Kernel + memory-copy traces of the pipelined `value` runs (tool): C5 x10 one rank, C4, C2 --
# where a pipelined step's time goes beside its kernels.  Each step bounded; a failure ends the run.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04t} && rm -rf $O && mkdir -p $O
P="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c5 -o kt --output-format csv \
  -- python3 bench.py --workload c5 --scale 10 --steps 20 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || { echo c5 failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c4 -o kt --output-format csv \
  -- python3 bench.py --steps 10 $P > $O/c4.log 2>&1 || { echo c4 failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c2 -o kt --output-format csv \
  -- python3 bench.py --workload c2 --steps 10 $P > $O/c2.log 2>&1 || { echo c2 failed; exit 1; }
find $O -name "*.csv" | xargs ls -la
