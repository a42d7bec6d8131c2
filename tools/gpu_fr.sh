#!/bin/bash
# frontier engine: GPU tests, then frontier vs DFS on the Drive profiling batch (+ kernel trace)
set -o pipefail
mkdir -p gpurun_out
export KETO_FR_VERBOSE=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_frontier.py tests/test_gpu_parity.py > gpurun_out/fr_tests.log 2>&1 || { tail -30 gpurun_out/fr_tests.log; exit 1; }
tail -2 gpurun_out/fr_tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/frprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/frprof -o frprof -- python3 -u tools/prof_check.py --workload drive --batches 0 --compare > gpurun_out/fr_drive.log 2>&1 || { tail -30 gpurun_out/fr_drive.log; exit 1; }
grep -E "KETO_FRONTIER|stats|identical" gpurun_out/fr_drive.log; grep "^\[frontier\]" gpurun_out/fr_drive.log | tail -1
python3 tools/rocpd_summary.py $(find gpurun_out/frprof -name "*results.db" | head -1) 8
if [ -f tools/ab/libketo_frprof.so ]; then
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=tools/ab/libketo_frprof.so timeout -k 10 300 python3 tools/fr_phases.py > gpurun_out/fr_phases.log 2>&1 && cat gpurun_out/fr_phases.log
fi
