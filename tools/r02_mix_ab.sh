#!/bin/bash
# Llama-2-7B (1 GPU) and the CP=8 critical-rank proxy with the mixed-tile q|k|v launch on / off
# (PICOTRON_GEMM_MIX), interleaved: bash tools/r02_mix_ab.sh <tag> [rounds]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02mix}; R=${2:-2}
for i in $(seq 1 $R); do
  for v in 1 0; do
    PICOTRON_GEMM_MIX=$v timeout -k 10 300 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_llama_$v$i.json 2> gpurun_out/${T}_llama_$v$i.err || { echo llama failed; tail gpurun_out/${T}_llama_$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${T}_llama_$v$i.json')); print('llama2-7b mix=$v', round(d['value']), round(d['mfu'],4), round(d['roofline']['frac'],3))"
  done
done
for v in 1 0; do
  PICOTRON_GEMM_MIX=$v timeout -k 10 300 python -u bench.py --cp-proxy 8 --model llama2-7b --seq 32768 --mbs 1 --steps 3 > gpurun_out/${T}_cp_$v.json 2> gpurun_out/${T}_cp_$v.err || { echo cpproxy failed; tail gpurun_out/${T}_cp_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_cp_$v.json')); print('cp8 proxy mix=$v', round(d['value']), round(d['critical_rank_layer_ms'],2))"
done
