set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "padded_head or attention" > $O.hd_kernels.log 2>&1 || { echo kernel tests failed; tail -50 $O.hd_kernels.log; exit 1; }
grep -E "passed|failed" $O.hd_kernels.log | tail -1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py > $O.hd_parallel.log 2>&1 || { echo parallel tests failed; tail -50 $O.hd_parallel.log; exit 1; }
grep -E "passed|failed" $O.hd_parallel.log | tail -1
