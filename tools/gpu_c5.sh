cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_partition.py tests/test_gpu_scale.py -k "partition or c5" -x -v --timeout 500 --timeout-method thread > gpurun_out/c5_tests.log 2>&1
rc=$?; tail -5 gpurun_out/c5_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --workload c5 --scale 10 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; tail -3 gpurun_out/bench_c5.log; exit $rc
