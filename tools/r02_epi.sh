#!/bin/bash
# epilogue A/B: GEMM parity tests, tools/epi_bench.py against older builds, then the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; OLD=${2:-tools/ab/old.so}; ONLY=${3:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u tools/epi_bench.py --old $OLD --rounds 3 ${ONLY:+--only $ONLY} > gpurun_out/${T}_epi.log 2>&1 || { echo epi failed; tail gpurun_out/${T}_epi.log; exit 1; }
grep median gpurun_out/${T}_epi.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_b$i.json 2>/dev/null || { echo "bench failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_b$i.json')); print('bench', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['frac'],3))"
done
