#!/bin/bash
# GPU suite; bench with the lm_head CE statistics (default) and without; kernel-trace profile (csv)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02e}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; tail -5 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
cut -c1-700 gpurun_out/${T}_bench.json
PICOTRON_CE_STATS=0 timeout -k 10 400 python -u bench.py --cpu-tokens 0 > gpurun_out/${T}_bench_nostats.json 2> gpurun_out/${T}_bench_nostats.err || { echo bench nostats failed; tail gpurun_out/${T}_bench_nostats.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_nostats.json
timeout -k 10 400 python -u bench.py --cpu-tokens 0 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err || { echo bench2 failed; tail gpurun_out/${T}_bench2.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
ls gpurun_out/${T}_prof
