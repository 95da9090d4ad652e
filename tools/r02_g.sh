#!/bin/bash
# full GPU suite + bench x2 + kernel stats (misc kernels folded: CE mean, embedding sort)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; tail -5 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-tokens 0 > gpurun_out/${T}_b$i.json 2>/dev/null || { echo "bench failed"; exit 1; }
  echo "$(cut -c1-230 gpurun_out/${T}_b$i.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python -u bench.py --steps 1 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
