set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
for b in 4 8 16; do
  timeout -k 10 120 python -u tools/attn_bench.py --B $b --model-path > $O.attn_B$b.log 2>&1 || { echo attn failed; tail $O.attn_B$b.log; exit 1; }
  echo "== B $b"; tail -6 $O.attn_B$b.log
done
timeout -k 10 120 python -u tools/attn_bench.py --B 8 --model-path --variant attn_pair=1,0 > $O.attn_B8_pair.log 2>&1 || { echo attn failed; tail $O.attn_B8_pair.log; exit 1; }
echo "== B 8 pair 1,0"; tail -8 $O.attn_B8_pair.log
