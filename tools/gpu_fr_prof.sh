#!/bin/bash
# kernel-trace summary of the frontier vs DFS comparison on the Drive profiling batch
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/frprof -o frprof -- python3 -u tools/prof_check.py --workload drive --batches 0 --compare > gpurun_out/fr_prof.log 2>&1 || { tail -30 gpurun_out/fr_prof.log; exit 1; }
tail -4 gpurun_out/fr_prof.log
f=$(find gpurun_out/frprof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -20
