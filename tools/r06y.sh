set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_gpu.py > $O.graph_tests.log 2>&1 || { echo tests failed; tail -30 $O.graph_tests.log; exit 1; }
grep -E "passed|failed" $O.graph_tests.log | tail -1
