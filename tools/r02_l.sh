#!/bin/bash
# kernel-level A/B of the transposed-weight dX (PICOTRON_WT=0/1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02l}
for f in 0 1; do
  PICOTRON_WT=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_wt$f -o p -- python -u bench.py --steps 1 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_wt$f.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_wt$f.log; exit 1; }
done
