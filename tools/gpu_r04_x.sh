#!/bin/bash
# Expand walk records + grid A/B, and the store probe in the bench's own context (tool).
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04x} && rm -rf $O && mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -k "xpand or tree or Tree" --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
A="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --steps 5"
for b in 8 16; do
  KETO_XW_BPC=$b KETO_PATCH_VERBOSE=1 timeout -k 10 400 python3 -u bench.py $A > $O/b$b.log 2>&1 || { echo "bench $b failed"; tail -5 $O/b$b.log; exit 1; }
  tail -1 $O/b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['expand']; print('bpc $b', 'api %.3f'%x['ms_per_batch'], 'kernel %.3f'%x['traversal_kernel_ms'], 'frac %.4f'%x['roofline']['frac'], 'patch', round(d['incremental_snapshot']['patch_ms'],1), round(d['incremental_snapshot']['new_objects']['patch_ms'],1), 'transact', round(d['incremental_snapshot']['transact_ms'],1))"
done
# config 5 one rank under the kernel trace (round-3 verdict: this command once died in static teardown)
rm -rf $O/c5kt && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5kt -o kt --output-format csv \
  -- python3 bench.py --workload c5 --scale 10 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5kt.log 2>&1
echo "c5 kernel trace rc=$?"; grep -ci "core\|segmentation\|SIGSEGV" $O/c5kt.log || true
cp $(find $O/c5kt -name "*kernel_stats.csv" | head -1) $O/c5_kernel_stats.csv 2>/dev/null
python3 tools/kt_batches.py $(find $O/c5kt -name "*kernel_trace.csv" | head -1) > $O/c5_batch_stats.txt 2>&1 || true
rm -rf $O/c5kt; head -14 $O/c5_batch_stats.txt
