#!/bin/bash
# d64 attention forward: waves per workgroup 2 / 8 vs 4, and causal pairing off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02t}
for nw in 2 8; do
  timeout -k 10 120 python -u tools/attn_bench.py --rounds 6 --old tools/ab/libattn_nw64_$nw.so > gpurun_out/${T}_nw$nw.log 2>&1 || { echo "nw $nw failed"; tail gpurun_out/${T}_nw$nw.log; exit 1; }
  echo "old = NW $nw:"; grep median gpurun_out/${T}_nw$nw.log
done
PICOTRON_ATTN_PAIR=0 timeout -k 10 120 python -u tools/attn_bench.py --rounds 4 > gpurun_out/${T}_nopair.log 2>&1 || { echo "nopair failed"; exit 1; }
echo "pair off:"; grep median gpurun_out/${T}_nopair.log
timeout -k 10 120 python -u tools/attn_bench.py --rounds 4 > gpurun_out/${T}_pair.log 2>&1 || { echo "pair failed"; exit 1; }
echo "pair on:"; grep median gpurun_out/${T}_pair.log
