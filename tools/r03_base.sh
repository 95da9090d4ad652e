#!/bin/bash
# round-3 baseline on the box: GPU suite, smoke, one bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03base}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],1), round(d['mfu'],4), round(d['roofline']['frac'],3))"
