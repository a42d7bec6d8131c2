#!/bin/bash
# HBM traffic of bench.py's dominant kernel, per launch, from two separate rocprofv3 --pmc
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass: MI355X_MICROARCH.md "rocprofv3 PMC
# slots").  Writes profiles/<round>_traffic_<workload>.json, which bench.py reports as
# roofline.traffic.   usage: tools/pmc_traffic.sh r01 c2
set -eu
cd "$(dirname "$0")/.."
ROUND=${1:-r01}
WL=${2:-c2}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic_$WL
mkdir -p $OUT profiles
ARGS="--workload $WL --steps 3 --warmup 0 --no-cpu-baseline --latency-iters 0 --serve-clients 0 --no-store-probe"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/parse_pmc.py $OUT $OUT/${ROUND}_traffic_$WL.json  # copy into profiles/ to commit
