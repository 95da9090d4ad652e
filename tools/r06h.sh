set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
bash tools/gpu.sh $1 envab A="PICOTRON_WGRAD_PAIR_DOWN=0" B="PICOTRON_WGRAD_PAIR_DOWN=1" ROUNDS=2 || exit 1
for pr in 0 1; do
  PICOTRON_WGRAD_PAIR_DOWN=$pr timeout -k 10 300 python -u bench.py --dp-bucket --grad-type fp32 --steps 3 --cpu-tokens 0 > $O.dp_fp32_down$pr.json 2>/dev/null || { echo dp failed; exit 1; }
  python -c "import json; d=json.load(open('$O.dp_fp32_down$pr.json')); print('dp fp32 pair_down $pr', round(d['value']), round(d['ms_per_step'],1))"
done
