#!/bin/bash
# whole-step A/B of two builds of libpicotron_hip.so (swapped in place), interleaved rounds, after the GPU tests of the new one
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; NEW=$2; OLD=$3; ROUNDS=${4:-2}
LIB=picotron_amd/lib/libpicotron_hip.so
cp $NEW $LIB
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in $(seq 1 $ROUNDS); do
  for v in new old; do
    if [ $v = new ]; then cp $NEW $LIB; else cp $OLD $LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_$v$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/${T}_$v$i.json')); print('$v', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['frac'],3))"
  done
done
cp $NEW $LIB
