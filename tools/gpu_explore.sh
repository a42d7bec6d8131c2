#!/bin/bash
# Exploration pass: C5 phase breakdown (closure levels, closure build phases) and C2 on the
# frontier engine vs the union interpreter.  Each GPU step has its own limit; the first failure
# ends the run.
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
KETO_PART_VERBOSE=1 KETO_BUILD_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 3 --warmup 1 \
  > gpurun_out/x_c5.log 2>&1
tail -1 gpurun_out/x_c5.log
timeout -k 10 300 python3 -u bench.py --workload c2 --serve-clients 0 --latency-iters 0 > gpurun_out/x_c2_union.log 2>&1
tail -1 gpurun_out/x_c2_union.log | cut -c1-400
KETO_UNION_FRONTIER=1 KETO_FR_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --workload c2 --serve-clients 0 --latency-iters 0 \
  > gpurun_out/x_c2_frontier.log 2>&1
tail -1 gpurun_out/x_c2_frontier.log | cut -c1-400
grep "^\[frontier\]" gpurun_out/x_c2_frontier.log | tail -2
