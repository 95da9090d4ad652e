set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in tools/ab/rebal.so tools/ab/head.so tools/ab/rebal.so tools/ab/head.so; do
  cp $f picotron_amd/lib/libpicotron_hip.so || exit 1
  echo "== $f"; timeout -k 10 200 python -u tools/gemm_kscan.py 2>/dev/null | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tile'],d['a_k'],d['b_k'],d['epi'],d['us'],d['intercept_us'],d['tflops_at_16k'])" || exit 1
done
cp tools/ab/rebal.so picotron_amd/lib/libpicotron_hip.so
