#!/bin/bash
# A/B (tool): the bench line of the current build and of every tools/ab lib on one workload.
#   usage: tools/ab_bench.sh [c4|c3|c2]
cd "$(dirname "$0")/.."
shopt -s nullglob
mkdir -p gpurun_out
WL=${1:-c4}
for lib in cur tools/ab/libketo_*.so; do
  if [ $lib = cur ]; then unset KETO_MI355X_LIB_OVERRIDE; else export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; fi
  timeout -k 10 240 python3 -u bench.py --workload $WL --steps 10 --no-cpu-baseline --latency-iters 100 ${AB_BENCH_ARGS:-} \
    > gpurun_out/ab_bench.log 2>&1 || { tail -3 gpurun_out/ab_bench.log; exit 1; }
  tail -1 gpurun_out/ab_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']/1e6,2), 'M/s kernel', round(d['roofline']['kernel_ms'],2), 'ms p99', round(d['p99_batch_latency_ms'],2), 'allowed', d['allowed_fraction'], 'expand_ms', d['expand'] and round(d['expand']['ms_per_batch'],2), 'serve', d['serving'] and (round(d['serving']['checks_per_s']), round(d['serving']['p99_request_ms'],1)))"
done
