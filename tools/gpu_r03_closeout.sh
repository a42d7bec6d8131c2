#!/bin/bash
# Round close-out on one box: smoke + the whole -m gpu suite (tools/gpu_r03_endcheck.sh), then
# the final measurements (tools/gpu_r03_final2.sh).  A failure ends the run.
set -u
cd "$(dirname "$0")/.."
bash tools/gpu_r03_endcheck.sh ${1:-r03z}_check || exit 1
bash tools/gpu_r03_final2.sh ${1:-r03z}
