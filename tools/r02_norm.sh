#!/bin/bash
# RMSNorm kernels: launch-config sweep of the new build vs the previous kernels (tools/ab/libnorm_old.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02n}
timeout -k 10 120 python -u tools/norm_bench.py --old tools/ab/libnorm_old.so > gpurun_out/${T}_norm.log 2>&1 || { echo norm bench failed; tail -30 gpurun_out/${T}_norm.log; exit 1; }
cat gpurun_out/${T}_norm.log
timeout -k 10 120 python -u tools/norm_bench.py --cols 4096 --rows 4096 --old tools/ab/libnorm_old.so > gpurun_out/${T}_norm4k.log 2>&1 || { echo norm bench 4k failed; tail -30 gpurun_out/${T}_norm4k.log; exit 1; }
cat gpurun_out/${T}_norm4k.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "norm or layer or model" > gpurun_out/${T}_pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/${T}_pytest.log
