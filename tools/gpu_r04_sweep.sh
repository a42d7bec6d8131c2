#!/bin/bash
# Random-world parity sweep on the GPU (tool): tools/parity_sweep.py over 2,000 seeds x 2 sizes x
# rewrites on/off with the engine's own choice (block engine for these small batches), then
# 1,000 seeds with the generation engine forced.
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/${1:-r04sw} && rm -rf $O && mkdir -p $O
timeout -k 10 500 python3 -u tools/parity_sweep.py --seeds 60:2060 > $O/auto.log 2>&1
rc=$?; tail -1 $O/auto.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
KETO_FR_ENGINE=gen timeout -k 10 400 python3 -u tools/parity_sweep.py --seeds 2060:3060 > $O/gen.log 2>&1
rc=$?; tail -1 $O/gen.log | cut -c1-400; exit $rc
