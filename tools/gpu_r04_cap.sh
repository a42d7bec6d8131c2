#!/bin/bash
# Generation-engine spawn cap A/B (tool): the frontier / parity / spine GPU tests and the
# generation-engine random-world sweep on the in-tree library (cap on), then bench.py's C4 and C3
# lines for in-tree vs tools/ab/libketo_nocap.so (KETO_FR_NOSPAWNCAP).
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04cap} && rm -rf $O && mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_spine.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
KETO_FR_ENGINE=gen timeout -k 10 400 python3 -u tools/parity_sweep.py --seeds 2060:3060 > $O/gen.log 2>&1
rc=$?; tail -1 $O/gen.log | cut -c1-500; [ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
for w in c4 c3; do for v in base nocap base nocap; do
  if [ $v = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$v.so; fi
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --workload $w $A > $O/$w.$v.log 2>&1 \
    || { echo "$w $v failed"; tail -5 $O/$w.$v.log; exit 1; }
  tail -1 $O/$w.$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; f=d['frontier']; print('$w $v', 'value %.1fM' % (d['value']/1e6), 'step %.3f' % d['ms_per_step'], 'resident kernel %.3f' % d['device_resident']['kernel_ms'], 'goals %.1fM gens %d' % (f['goals_per_batch']/1e6, f['generations_max']), 'mism', p['mismatches'])"
done; done
