#!/bin/bash
# The other BASELINE configs on one GPU: Llama-2-7B (32 layers, mbs 4 seq 1024), the TP=8 per-rank
# compute proxy (SmolLM-1.7B shards) and the CP=8 critical-rank proxy (Llama-2-7B at 32k)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02cfg}
timeout -k 10 400 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_llama.json 2> gpurun_out/${T}_llama.err || { echo llama failed; tail gpurun_out/${T}_llama.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_llama.json')); print('llama2-7b', round(d['value']), round(d['mfu'],4), round(d['roofline']['frac'],3))"
timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 3 > gpurun_out/${T}_tpproxy.json 2> gpurun_out/${T}_tpproxy.err || { echo tpproxy failed; tail gpurun_out/${T}_tpproxy.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_tpproxy.json')); print('tp8 proxy', round(d['value']), round(d['ms_per_microbatch'],2), round(d['roofline']['frac'],3))"
timeout -k 10 300 python -u bench.py --cp-proxy 8 --model llama2-7b --seq 32768 --mbs 1 --steps 3 > gpurun_out/${T}_cpproxy.json 2> gpurun_out/${T}_cpproxy.err || { echo cpproxy failed; tail gpurun_out/${T}_cpproxy.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_cpproxy.json')); print('cp8 proxy', round(d['value']), round(d['critical_rank_layer_ms'],2), round(d['roofline']['fwd_frac'],3), round(d['roofline']['bwd_frac'],3))"
