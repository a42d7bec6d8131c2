#!/bin/bash
# Patch-timing variance (tool): bench.py's C4 store probe twice, each in its own process, with the
# patcher's per-phase timing on stderr (KETO_PATCH_VERBOSE).
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04pt} && rm -rf $O && mkdir -p $O
for r in ${RUNS:-1 2}; do
  KETO_PATCH_VERBOSE=1 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 2 --warmup 1 > $O/run$r.log 2>&1 \
    || { echo "run $r failed"; tail -5 $O/run$r.log; exit 1; }
  grep -E "keto patch|store probe" $O/run$r.log | head -40
  tail -1 $O/run$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); i=d['incremental_snapshot']; print('run $r patch', round(i['patch_ms'],1), 'new files', round(i['new_objects']['patch_ms'],1))"
done
