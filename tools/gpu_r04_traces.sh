#!/bin/bash
# Kernel traces of the pipelined `value` runs (tool): C2 and C4 -- the async batches' kernels and
# the gaps between them, beside the device-resident batches of the same run.  (--memory-copy-trace
# is left out: with it rocprofv3's own teardown faults at exit and no trace is written)
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04t} && rm -rf $O && mkdir -p $O
P="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for w in c2 c4; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O/$w -o kt --output-format csv -- python3 bench.py --workload $w --steps 10 $P > $O/$w.log 2>&1 \
    || { echo "$w failed"; tail -3 $O/$w.log; exit 1; }
  cp $(find $O/$w -name "*kernel_trace.csv" | head -1) $O/${w}_kernel_trace.csv && rm -rf $O/$w
done
ls -la $O
