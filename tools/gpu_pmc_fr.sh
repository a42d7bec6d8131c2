#!/bin/bash
# PMC passes over one frontier batch (Drive profiling workload): SQ issue counters, HBM bytes
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
P="python3 tools/prof_check.py --workload drive --batches 1"
rm -rf gpurun_out/pmcfr_*
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmcfr_sq -o pmc --output-format csv -- $P > gpurun_out/pmcfr_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcfr_fetch -o pmc --output-format csv -- $P > gpurun_out/pmcfr_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcfr_write -o pmc --output-format csv -- $P > gpurun_out/pmcfr_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_INSTS_SMEM -d gpurun_out/pmcfr_tcc -o pmc --output-format csv -- $P > gpurun_out/pmcfr_tcc.log 2>&1 || exit $?
python3 tools/pmc_kernels.py gpurun_out/pmcfr_sq gpurun_out/pmcfr_fetch gpurun_out/pmcfr_write gpurun_out/pmcfr_tcc 2>&1 | head -60
