#!/bin/bash
# frontier diagnosis on the Drive profiling batch: phase profile (KETO_FR_PROF build) and the
# PMC passes of tools/gpu_pmc_fr.sh.  Each GPU step has its own limit; a failure ends the run.
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
KETO_FR_VERBOSE=1 KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_frprof.so timeout -k 10 200 python3 tools/fr_phases.py > gpurun_out/fr_phases.log 2>&1 || { tail -5 gpurun_out/fr_phases.log; exit 1; }
grep -v "^\[frontier\]" gpurun_out/fr_phases.log; grep "^\[frontier\]" gpurun_out/fr_phases.log | tail -1
bash tools/gpu_pmc_fr.sh
