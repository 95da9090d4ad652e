#!/bin/bash
# attention A/B: this build vs tools/ab/libattn_old.so (graph-timed, same process), then the GPU suite's attention tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02at}
timeout -k 10 120 python -u tools/attn_bench.py --rounds 6 --old tools/ab/libattn_old.so > gpurun_out/${T}_d64.log 2>&1 || { echo attn d64 failed; tail -30 gpurun_out/${T}_d64.log; exit 1; }
cat gpurun_out/${T}_d64.log
timeout -k 10 120 python -u tools/attn_bench.py --rounds 6 --B 1 --S 4096 --D 128 --old tools/ab/libattn_old.so > gpurun_out/${T}_d128.log 2>&1 || { echo attn d128 failed; tail -30 gpurun_out/${T}_d128.log; exit 1; }
cat gpurun_out/${T}_d128.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or ring or layer or model or shapes or golden or api" > gpurun_out/${T}_pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/${T}_pytest.log
