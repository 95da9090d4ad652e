set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 300 python -u tools/attn_bench.py --rounds 4 --old tools/ab/base.so,tools/ab/attn_pair.so --variant attn_pair=0,1 > $O.attn_d64.log 2>&1 || { echo attn failed; tail -30 $O.attn_d64.log; exit 1; }
grep -E "median|rel" $O.attn_d64.log
