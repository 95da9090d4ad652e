set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "norm" > gpurun_out/r03d_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/norm_bench.py --old tools/ab/libnorm_base.so > gpurun_out/r03d_norm.log 2>&1 && \
timeout -k 10 300 python -u tools/norm_bench.py --old tools/ab/libnorm_base.so >> gpurun_out/r03d_norm.log 2>&1
