#!/bin/bash
# Round-4 C4 A/B (tool, not product): the in-tree library and tools/ab/libketo_<name>.so variants on
# bench.py's own C4 batch (probes off) -- ms/step, check-path ms -- and one PMC pass each of the L2
# requests (TCC_HIT_sum + TCC_MISS_sum) per kernel.  A failing step ends the run.
#   usage: tools/gpu_r04_ab.sh OUTDIR [name ...]
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
OUT=$1; shift; mkdir -p $OUT
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for name in base "$@"; do
  if [ $name = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$name.so; fi
  export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib
  timeout -k 10 300 python3 -u bench.py $ARGS > $OUT/ab_$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/ab_$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value %.1fM' % (d['value']/1e6), 'ms/step %.3f' % d['ms_per_step'], 'resident kernel %.3f' % d['roofline']['kernel_ms'], 'goals', d.get('frontier',{}).get('goals_per_batch'), 'gens', d.get('frontier',{}).get('generations_max'), 'mism', d['pipeline'].get('mismatches'))" $OUT/ab_$name.log $name
  if [ "${PMC:-1}" = 1 ]; then
    timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc_$name -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 0 $ARGS > $OUT/tcc_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
  fi
done
