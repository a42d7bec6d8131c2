#!/bin/bash
# C4 A/B: the in-tree library and each tools/ab/libketo_<name>.so named on the command line, on
# bench.py's own C4 batch (probes off): ms/step, check-path ms, goals; with PMC=1 also the
# FETCH_SIZE / WRITE_SIZE passes of each (tools/parse_pmc.py).  A failing step ends the run.
#   usage: tools/gpu_c4_ab.sh [name ...]
set -u
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for name in base "$@"; do
  if [ $name = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$name.so; fi
  export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib
  timeout -k 10 300 python3 -u bench.py $ARGS > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ab_$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms/step %.3f' % d['ms_per_step'], 'kernel %.3f' % d['roofline']['kernel_ms'], 'goals', d.get('frontier',{}).get('goals_per_batch'), 'gens', d.get('frontier',{}).get('generations_max'))" gpurun_out/ab_$name.log $name
  if [ "${PMC:-0}" = 1 ]; then
    O=gpurun_out/ab_pmc_$name; mkdir -p $O
    P="--steps 3 --warmup 0 $ARGS"
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python3 bench.py $P > $O/fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python3 bench.py $P > $O/write.log 2>&1 || { echo "pmc write failed"; exit 1; }
    python3 tools/parse_pmc.py $O $O/traffic.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  traffic GB/batch: fetch %.2f write %.2f total %.2f' % (d['fetch_bytes_per_launch']/1e9, d['write_bytes_per_launch']/1e9, d['traffic_bytes_per_launch']/1e9))"
  fi
done
