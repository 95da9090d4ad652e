set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_d.so --rounds 6 > gpurun_out/r03c_pair1.log 2>&1 && \
PICOTRON_ATTN_PAIR=0 timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_d.so --rounds 6 > gpurun_out/r03c_pair0.log 2>&1
