#!/bin/bash
# Small expand-subject A/B (tool): the frontier / parity GPU tests on the in-tree library (small-ES on, oracle with
# it), then bench.py's C4 and C3 lines for in-tree vs tools/ab/libketo_nosmall.so.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04sm} && rm -rf $O && mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_spine.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for w in c4 c3; do for v in base nosmall base nosmall; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --workload $w $A > $O/$w.$v.log 2>&1 \
    || { echo "$w $v failed"; tail -5 $O/$w.$v.log; exit 1; }
  tail -1 $O/$w.$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; f=d['frontier']; print('$w $v', 'value %.1fM' % (d['value']/1e6), 'step %.3f' % d['ms_per_step'], 'resident kernel %.3f' % d['device_resident']['kernel_ms'], 'goals %.1fM gens %d' % (f['goals_per_batch']/1e6, f['generations_max']), 'mism', p['mismatches'])"
done; done
