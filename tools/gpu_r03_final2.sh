#!/bin/bash
# Final measurements of this build: the C4 traffic profile (sha-stamped, tools/pmc_traffic.sh), the
# default C4 bench line that reports it, and the config-5 line (C3 x10, one rank, with its CPU
# baseline).  Each step bounded; a failure ends the run.   usage: tools/gpu_r03_final2.sh [tag]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03g} && rm -rf $O && mkdir -p $O
bash tools/pmc_traffic.sh r03 c4 || { echo "pmc traffic failed"; exit 1; }
cp gpurun_out/pmc_traffic_c4/r03_traffic_c4.json $O/ && cp $O/r03_traffic_c4.json profiles/
timeout -k 10 600 python3 -u bench.py > $O/bench_c4.log 2>&1 || { echo "c4 bench failed"; tail -8 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log > $O/bench_c4.json
timeout -k 10 400 python3 -u bench.py --workload c5 --scale 10 --steps 10 --warmup 2 > $O/bench_c5.log 2>&1 \
  || { echo "c5 bench failed"; tail -8 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log > $O/bench_c5.json
cut -c1-400 $O/bench_c4.json; cut -c1-400 $O/bench_c5.json
