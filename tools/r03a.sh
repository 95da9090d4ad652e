set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" tests/test_api_gpu.py tests/test_model_gpu.py > gpurun_out/r03a_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_base.so --rounds 6 > gpurun_out/r03a_d64.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_base.so --rounds 4 --B 1 --S 4096 --D 128 > gpurun_out/r03a_d128.log 2>&1
