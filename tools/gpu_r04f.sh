cd /root/repo && export TMPDIR=/tmp && D=gpurun_out/r04f && mkdir -p $D
ARGS="--no-cpu-baseline --serve-clients 0 --latency-iters 0 --no-store-probe --steps 3 --warmup 0"
timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum -d $D/tcp -o pmc --output-format csv -- python3 bench.py $ARGS > $D/tcp.log 2>&1 || { echo tcp failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_BUSY_avr TD_BUSY_avr -d $D/tcp2 -o pmc --output-format csv -- python3 bench.py $ARGS > $D/tcp2.log 2>&1 || echo tcp2 failed
KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_frprof.so timeout -k 10 300 python3 tools/fr_phases.py --c4 > $D/phases.txt 2>&1; echo phases rc=$?
cat $D/phases.txt | tail -8
