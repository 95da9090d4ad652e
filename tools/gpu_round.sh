#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace (+ optional PMC passes).
# Usage (from the repo root, on the box): bash tools/gpu_round.sh <tag> [pmc]
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest rc=$?" | tee -a gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o k -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo prof failed; exit 1; }
gzip -f gpurun_out/${TAG}_prof/k_kernel_trace.csv
if [ "$2" = "pmc" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc1 -o f -- python -u bench.py --steps 1 --warmup 0 --grad-acc 1 --cpu-tokens 0 --no-probe > gpurun_out/${TAG}_pmc1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc2 -o w -- python -u bench.py --steps 1 --warmup 0 --grad-acc 1 --cpu-tokens 0 --no-probe > gpurun_out/${TAG}_pmc2.log 2>&1 || exit 1
fi
find gpurun_out -name "*.db" -delete
tail -1 gpurun_out/${TAG}_bench.log
