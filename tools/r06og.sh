set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_api_gpu.py > $O.ce_tests.log 2>&1 || { echo tests failed; tail -50 $O.ce_tests.log; exit 1; }
grep -E "passed|failed" $O.ce_tests.log | tail -1
