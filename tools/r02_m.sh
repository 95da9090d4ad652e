#!/bin/bash
# RMSNorm backward: launch shape x next-row prefetch sweep (one process per PT_NORM value)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02m}
: > gpurun_out/${T}_norm.log
for cfg in "4,4,8,2,0" "4,4,8,1,1" "4,4,8,1,0" "4,4,4,2,1" "4,4,8,2,0"; do
  PT_NORM=$cfg timeout -k 10 100 python -u tools/norm_bench.py >> gpurun_out/${T}_norm.log 2>&1 || { echo "norm $cfg failed"; tail gpurun_out/${T}_norm.log; exit 1; }
done
grep cfg gpurun_out/${T}_norm.log
