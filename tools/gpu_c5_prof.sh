#!/bin/bash
# Where a config-5 batch's time goes (one rank, C3 x<scale>): the bench line with the builder's
# and the closure's phase times, then a kernel trace of the same run (no counters).
#   usage: tools/gpu_c5_prof.sh tag [scale]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5p} && rm -rf $O && mkdir -p $O
S=${2:-10}
ARGS="--workload c5 --scale $S --steps 10 --warmup 2 --no-cpu-baseline"
[ -n "${SKIP_LINE:-}" ] || KETO_BUILD_VERBOSE=1 KETO_PART_VERBOSE=1 timeout -k 10 400 python3 -u bench.py $ARGS > $O/c5.log 2>&1 \
  || { echo "c5 bench failed"; tail -8 $O/c5.log; exit 1; }
grep -E "keto (build|partition)" $O/c5.log | tail -45
grep '^{' $O/c5.log | cut -c1-700
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 \
  --output-format csv -- python3 bench.py $ARGS > $O/prof.log 2>&1 || { echo "profile failed"; tail -8 $O/prof.log; exit 1; }
for f in $(find $O/prof -name "*_stats.csv"); do echo "== $f"; head -25 $f | cut -c1-200; done
exit 0
