#!/bin/bash
# The GPU-box drivers the docs cite (tool, not product), one subcommand per kind of run; every
# GPU step is bounded by its own timeout and a failing step ends the run.
#   tools/gpu_round.sh OUT tests              the -m gpu suite (pytest, one process)
#   tools/gpu_round.sh OUT bench [args]       bench.py's line (default: C4 on one GPU)
#   tools/gpu_round.sh OUT profile [args]     rocprofv3 --kernel-trace --stats of bench.py, summarised
#   tools/gpu_round.sh OUT traffic [wl]       HBM bytes per launch of the dominant kernel: FETCH_SIZE and
#                                             WRITE_SIZE in separate --pmc passes (tools/parse_pmc.py)
#   tools/gpu_round.sh OUT ab name...         bench.py with the in-tree library and tools/ab/libketo_<name>.so
#                                             (tools/ab_build.sh), probes off
#   tools/gpu_round.sh OUT gentime v...       bench.py per variant (base | rootk | nostash | an ab library name) with
#                                             KETO_FR_GENTIME: the line and the median time of each generation
#   tools/gpu_round.sh OUT sq [wl]            SQ / TCC counters per kernel of the check path (two --pmc passes,
#                                             tools/pmc_split.py): issue vs wait, instructions per batch
#   tools/gpu_round.sh OUT sqlds [wl]         per-generation LDS / wait / instruction-mix counters of fr_expand (pmc_gens.py)
#   tools/gpu_round.sh OUT patch              the store probe alone, the patcher's phase times (KETO_PATCH_VERBOSE)
#   tools/gpu_round.sh OUT c5 [scale]         tests/test_gpu_c5.py (8 gloo ranks sharing the GPU) and the C5
#                                             bench rehearsal at that scale (default 40 / 10)
#   tools/gpu_round.sh OUT sweep              the random-world parity sweep (tools/parity_sweep.py)
#   tools/gpu_round.sh OUT exitprobe MODE     tools/exit_probe.py under --kernel-trace --memory-copy-trace
#                                             (last step of a call: it may end in a signal at exit)
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
OUT=gpurun_out/$1; CMD=$2; shift 2
mkdir -p $OUT
QUIET="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe"
line() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); f=d.get('frontier') or {}; print(sys.argv[2], 'value %.1fM' % (d['value']/1e6), 'ms/step %.3f' % d['ms_per_step'], 'check path %s ms' % d['roofline'].get('kernel_ms'), 'goals', f.get('goals_per_batch'), 'gens', f.get('generations_max'))" "$1" "$2"; }
case $CMD in
tests)
  timeout -k 10 1300 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; exit $rc ;;
bench)
  timeout -k 10 900 python3 -u bench.py "$@" > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
  line $OUT/bench.log bench ;;
profile)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 $QUIET "$@" \
    > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
  python3 tools/rocpd_summary.py $(find $OUT/prof -name "*results.db" | head -1) 25 | tee $OUT/kernel_summary.txt ;;
traffic)
  WL=${1:-c4}; A="--workload $WL --steps 3 --warmup 0 $QUIET"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 bench.py $A > $OUT/fetch.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 bench.py $A > $OUT/write.log 2>&1 || exit 1
  python3 tools/parse_pmc.py $OUT $OUT/traffic_$WL.json ;;
ab)
  for name in base "$@"; do
    if [ $name = base ]; then lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; else lib=$PWD/tools/ab/libketo_$name.so; fi
    KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $QUIET \
      > $OUT/ab_$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/ab_$name.log; exit 1; }
    line $OUT/ab_$name.log $name
  done ;;
gentime)
  for name in "$@"; do
    lib=$PWD/djy-keto_amd/keto_mi355x/libketo_mi355x.so; env=""
    case $name in base) ;; rootk) env="KETO_FR_ROOT_KERNEL=1" ;; nostash) env="KETO_FR_NOSTASH=1" ;;
      *) lib=$PWD/tools/ab/libketo_$name.so ;; esac
    env $env KETO_FR_GENTIME=1 KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$lib timeout -k 10 300 \
      python3 -u bench.py --steps 10 --warmup 3 $QUIET > $OUT/gt_$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/gt_$name.log; exit 1; }
    line $OUT/gt_$name.log $name; python3 tools/gentime.py $OUT/gt_$name.log
  done ;;
sq)
  WL=${1:-c4}; A="--workload $WL --steps 3 --warmup 0 $QUIET"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    -d $OUT/sq1 -o pmc --output-format csv -- python3 bench.py $A > $OUT/sq1.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum \
    -d $OUT/sq2 -o pmc --output-format csv -- python3 bench.py $A > $OUT/sq2.log 2>&1 || exit 1
  python3 tools/pmc_split.py $OUT/sq_$WL.json $OUT/sq1 $OUT/sq2 | cut -c1-400 | head -12 ;;
sqlds)
  WL=${1:-c4}; A="--workload $WL --steps 3 --warmup 0 $QUIET"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    -d $OUT/lds1 -o pmc --output-format csv -- python3 bench.py $A > $OUT/lds1.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA \
    -d $OUT/lds2 -o pmc --output-format csv -- python3 bench.py $A > $OUT/lds2.log 2>&1 || exit 1
  python3 tools/pmc_gens.py $OUT/lds1 $OUT/lds2 | cut -c1-400 ;;
patch)
  KETO_PATCH_VERBOSE=1 timeout -k 10 400 python3 -u tools/patch_probe.py 10 > $OUT/patch.log 2>&1 || { tail -5 $OUT/patch.log; exit 1; }
  grep -E "keto (patch|advance)|advance_ms" $OUT/patch.log | cut -c1-900 | head -60 ;;
c5)
  S=${1:-40}; B=${2:-10}
  KETO_C5_SCALE=$S timeout -k 10 1100 python3 -u -m pytest -x -v -s --timeout 1080 --timeout-method thread tests/test_gpu_c5.py \
    > $OUT/c5test.log 2>&1 || { grep -E "failed|Error" $OUT/c5test.log | head; exit 1; }
  cp gpurun_out/c5x${S}*_phases.json $OUT/ 2>/dev/null; true
  KETO_BENCH_BACKEND=gloo KETO_POOL_CAP_MB=1 KETO_SCRATCH_CAP_MB=1 KETO_PART_TRIM=1 timeout -k 10 900 \
    python3 -u bench.py --workload c5 --scale $B --gpus 8 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c5bench.log 2>&1 \
    || { tail -5 $OUT/c5bench.log; exit 1; }
  line $OUT/c5bench.log c5 ;;
sweep)
  timeout -k 10 600 python3 -u tools/parity_sweep.py --seeds ${1:-60:2060} > $OUT/sweep.log 2>&1; rc=$?; tail -1 $OUT/sweep.log | cut -c1-600; exit $rc ;;
exitprobe)
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/mct -o kt --output-format csv -- python3 tools/exit_probe.py ${1:-async} \
    > $OUT/exit_${1:-async}.log 2>&1
  rc=$?; echo "exit_probe ${1:-async} rc=$rc"; tail -3 $OUT/exit_${1:-async}.log; exit $rc ;;
*) echo "unknown subcommand $CMD"; exit 2 ;;
esac
