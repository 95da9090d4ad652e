#!/bin/bash
# round-2 evidence on the current tree: GPU suite, default bench line, kernel-trace summary, TP/CP proxies
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02z}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; tail -5 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 3 > gpurun_out/${T}_tpproxy.json 2> gpurun_out/${T}_tpproxy.err || { echo tpproxy failed; tail gpurun_out/${T}_tpproxy.err; exit 1; }
timeout -k 10 300 python -u bench.py --cp-proxy 8 --model llama2-7b --seq 32768 --mbs 1 --steps 3 > gpurun_out/${T}_cpproxy.json 2> gpurun_out/${T}_cpproxy.err || { echo cpproxy failed; tail gpurun_out/${T}_cpproxy.err; exit 1; }
cut -c1-300 gpurun_out/${T}_tpproxy.json gpurun_out/${T}_cpproxy.json
timeout -k 10 400 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_llama.json 2> gpurun_out/${T}_llama.err || { echo llama failed; tail gpurun_out/${T}_llama.err; exit 1; }
cut -c1-300 gpurun_out/${T}_llama.json
