#!/bin/bash
# C3 bench line with the Expand and serving probes, then a two-rank rehearsal of the
# multi-GPU bench path (gloo, both ranks on the box's one GPU).  First failure ends the run.
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --workload c3 --steps 5 --no-cpu-baseline --serve-seconds 2 \
  > gpurun_out/bench_c3.log 2>&1
tail -1 gpurun_out/bench_c3.log
KETO_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29577 bench.py --workload c2 --gpus 2 --steps 5 --serve-clients 0 \
  > gpurun_out/bench_n2.log 2>&1
tail -1 gpurun_out/bench_n2.log
