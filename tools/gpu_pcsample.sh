#!/bin/bash
# PC sampling of the check path (tool): a -g build of frontier.hip (tools/ab/libketo_dbg.so) under
# rocprofv3's stochastic PC sampler on a short C4 bench; the samples are summed per source line
# and per instruction by tools/pcs_summary.py.   usage: tools/gpu_pcsample.sh [tag] [kernel regex]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-pcs} && rm -rf $O && mkdir -p $O
RX=${2:-fr_expand}
export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_dbg.so
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 3 --warmup 1 --no-store-probe"
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-65536} --kernel-include-regex "$RX" \
  -d $O/raw -o pcs --output-format csv -- python3 bench.py $ARGS > $O/run.log 2>&1
rc=$?; tail -5 $O/run.log
[ $rc -ne 0 ] && exit $rc
f=$(find $O/raw -name "*pc_sampling*.csv" | head -1); ls -la $(dirname "$f")
python3 tools/pcs_summary.py "$f" > $O/summary.txt && head -70 $O/summary.txt
rm -rf $O/raw
