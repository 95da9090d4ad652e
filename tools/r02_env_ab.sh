#!/bin/bash
# whole-step A/B of two environment settings (e.g. PICOTRON_DUAL_LM=0 vs 1), interleaved rounds,
# after the given GPU test files
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; A=$2; B=$3; ROUNDS=${4:-3}; TESTS=${5:-tests/test_model_gpu.py}
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_$v$i.json 2>/dev/null || { echo "bench $E failed"; exit 1; }
    [ $(wc -l < gpurun_out/${T}_$v$i.json) = 1 ] || echo "stdout has more than one line"
    python -c "import json,sys; d=json.load(open('gpurun_out/${T}_$v$i.json')); print('$E', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['frac'],3))"
  done
done
