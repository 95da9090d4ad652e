#!/bin/bash
# Llama-2-7B (1 GPU, ga 8) with several builds of libpicotron_hip.so swapped in place, interleaved:
#   bash tools/r02_llama_ab.sh <tag> <lib1,lib2,...> [rounds]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; IFS=, read -ra L <<< "$2"; R=${3:-2}
LIB=picotron_amd/lib/libpicotron_hip.so
[ $(md5sum "${L[@]}" | cut -d' ' -f1 | sort -u | wc -l) -eq ${#L[@]} ] || { echo "identical or missing builds in $2"; exit 1; }
for i in $(seq 1 $R); do
  for f in "${L[@]}"; do
    cp "$f" $LIB || exit 1
    n=$(basename $f .so)
    timeout -k 10 300 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_${n}_$i.json 2> gpurun_out/${T}_${n}_$i.err || { echo "llama $n failed"; tail gpurun_out/${T}_${n}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${T}_${n}_$i.json')); print('$n', round(d['value']), round(d['mfu'],4), round(d['roofline']['frac'],3))"
  done
done
cp "${L[0]}" $LIB
