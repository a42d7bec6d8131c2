cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/flake
T="tests/test_gpu_frontier.py::test_random_worlds_frontier_vs_oracle"
for i in 1 2 3; do timeout -k 10 120 python3 -m pytest -q -x --timeout 100 "$T[3-1024-False]" 2>&1 | tail -1; done
KETO_FR_ENGINE=block timeout -k 10 300 python3 -m pytest -q --timeout 280 tests/test_gpu_frontier.py -k random_worlds 2>&1 | tail -3
KETO_FR_ENGINE=gen timeout -k 10 300 python3 -m pytest -q --timeout 280 tests/test_gpu_frontier.py -k random_worlds 2>&1 | tail -3
