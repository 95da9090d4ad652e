set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_base.so,tools/ab/libattn_a.so --rounds 6 > gpurun_out/r03b_d64.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --old tools/ab/libattn_base.so,tools/ab/libattn_a.so --rounds 3 --B 1 --S 4096 --D 128 > gpurun_out/r03b_d128.log 2>&1
