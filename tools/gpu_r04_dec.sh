#!/bin/bash
# Block-engine repeat check without a decisive-key cap (tool): the frontier / parity / spine GPU
# tests, then the random-world sweep (tools/parity_sweep.py) over the seeds that found the cap,
# with the generation engine forced over 1,000 more, and 300 spine worlds x 3 width limits.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04dec} && rm -rf $O && mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_spine.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
timeout -k 10 500 python3 -u tools/parity_sweep.py --seeds 60:2060 > $O/auto.log 2>&1
rc=$?; tail -1 $O/auto.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
KETO_FR_ENGINE=gen timeout -k 10 400 python3 -u tools/parity_sweep.py --seeds 2060:3060 > $O/gen.log 2>&1
rc=$?; tail -1 $O/gen.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/parity_sweep.py --kind spine --seeds 100:400 > $O/spine.log 2>&1
rc=$?; tail -1 $O/spine.log | cut -c1-600; exit $rc
