#!/bin/bash
# Kernel-trace A/B on bench.py's C4 batch (probes off): per-kernel time of the in-tree library and
# of each tools/ab/libketo_<name>.so named (tools/kt_summary.py).  A failing step ends the run.
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --serve-clients 0 --latency-iters 0"
for name in base "$@"; do
  if [ $name = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$name.so; fi
  export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib
  rm -rf gpurun_out/kt_ab_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_ab_$name -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/kt_ab_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/kt_ab_$name.log; exit 1; }
  f=$(find gpurun_out/kt_ab_$name -name "*kernel_trace.csv" | head -1)
  echo "== $name"; python3 tools/kt_summary.py "$f" | grep -E "fr_|check_kernel|resolve|kernel,grid" | head -12
done
