set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_golden_gpu.py -k "g11 and (2-1-1)" > $O.g11_tests.log 2>&1 || { echo tests failed; tail -30 $O.g11_tests.log; exit 1; }
grep -E "max rel dev|passed|failed" $O.g11_tests.log | tail -4
