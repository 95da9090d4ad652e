set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_parallel_gpu.py -k "paired or golden or G8 or g8 or data_parallel or dp_bucket or loss_curve" -m gpu -x -q --timeout 300 --timeout-method thread > $O.pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error|assert" $O.pytest.log | head -20; exit 1; }
tail -1 $O.pytest.log
bash tools/gpu.sh $1 envab A="PICOTRON_WGRAD_PAIR=0" B="PICOTRON_WGRAD_PAIR=1" ROUNDS=2 || exit 1
for pr in 1 0; do
  PICOTRON_WGRAD_PAIR=$pr timeout -k 10 300 python -u bench.py --dp-bucket --grad-type fp32 --steps 3 --cpu-tokens 0 > $O.dp_fp32_pair$pr.json 2>/dev/null || { echo dp failed; exit 1; }
  python -c "import json; d=json.load(open('$O.dp_fp32_pair$pr.json')); print('dp fp32 pair $pr', round(d['value']), round(d['ms_per_step'],1))"
done
