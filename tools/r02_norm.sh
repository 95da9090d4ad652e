#!/bin/bash
# RMSNorm A/B: norm parity tests, then tools/norm_bench.py per PT_NORM launch shape against an older build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; OLD=${2:-tools/ab/head.so}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "rmsnorm or norm or layer" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for cfg in "4,4,8,2" "4,4,16,1" "4,4,8,2"; do
  PT_NORM=$cfg timeout -k 10 120 python -u tools/norm_bench.py --old $OLD > gpurun_out/${T}_norm_$cfg.log 2>&1 || { echo norm failed; tail gpurun_out/${T}_norm_$cfg.log; exit 1; }
  echo "== $cfg"; cat gpurun_out/${T}_norm_$cfg.log | grep -v "^$" | tail -3
done
