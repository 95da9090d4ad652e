#!/bin/bash
# whole-step A/B of builds of libpicotron_hip.so (swapped in place; the libs must travel to the box,
# so keep them out of .gpurunignore), interleaved rounds, after the GPU tests of the first one.
#   bash tools/r02_ab_bench.sh <tag> <lib1,lib2[,lib3...]> [rounds]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; LIBS=$2; ROUNDS=${3:-2}
LIB=picotron_amd/lib/libpicotron_hip.so
IFS=, read -ra L <<< "$LIBS"
for f in "${L[@]}"; do [ -f "$f" ] || { echo "missing $f on the box"; exit 1; }; done
[ $(md5sum "${L[@]}" | cut -d' ' -f1 | sort -u | wc -l) -eq ${#L[@]} ] || { echo "identical builds in $LIBS"; exit 1; }
cp "${L[0]}" $LIB || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in $(seq 1 $ROUNDS); do
  for f in "${L[@]}"; do
    cp "$f" $LIB || exit 1
    n=$(basename $f .so)
    timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_${n}_$i.json 2>/dev/null || { echo "bench $n failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/${T}_${n}_$i.json')); print('$n', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['frac'],3))"
  done
done
cp "${L[0]}" $LIB
