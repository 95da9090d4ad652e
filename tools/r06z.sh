set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "paired" > $O.pair_tests.log 2>&1 || { echo tests failed; tail -30 $O.pair_tests.log; exit 1; }
grep -E "passed|failed" $O.pair_tests.log | tail -1
