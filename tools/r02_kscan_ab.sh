#!/bin/bash
# tools/gemm_kscan.py for several builds (swapped in place, interleaved): bash tools/r02_kscan_ab.sh lib1.so,lib2.so [rounds]
set -o pipefail
export TMPDIR=/tmp
IFS=, read -ra L <<< "$1"; R=${2:-2}
[ $(md5sum "${L[@]}" | cut -d' ' -f1 | sort -u | wc -l) -eq ${#L[@]} ] || { echo "identical or missing builds in $1"; exit 1; }
for i in $(seq 1 $R); do
  for f in "${L[@]}"; do
    cp $f picotron_amd/lib/libpicotron_hip.so || exit 1
    echo "== $f"; timeout -k 10 200 python -u tools/gemm_kscan.py 2>/dev/null | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tile'],d['a_k'],d['b_k'],d['epi'],d['us'],d['intercept_us'],d['tflops_at_16k'])" || exit 1
  done
done
cp ${L[0]} picotron_amd/lib/libpicotron_hip.so
