#!/bin/bash
# Expand in parts (tool): the Expand GPU tests, then bench.py's expand probe on C4 with
# KETO_XW_PARTS=1 (one piece) and 2 / 4 (output copied part by part while the walk proceeds).
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04xz} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -k "xpand or tree or Tree" --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 5 --no-store-probe"
for z in 1 2 4 1 2 4; do
  KETO_XW_PARTS=$z timeout -k 10 400 python3 -u bench.py $A > $O/z$z.log 2>&1 || { echo "bench $z failed"; tail -5 $O/z$z.log; exit 1; }
  tail -1 $O/z$z.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['expand']; print('parts $z', 'api %.3f'%x['ms_per_batch'], 'pageable %.3f'%x['ms_per_batch_pageable_out'], 'walk %.3f'%x['traversal_kernel_ms'], 'frac %.4f'%x['roofline']['frac'], 'err', x['errors'], 'nodes', x['nodes_per_batch'])"
done
