set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "key_split" > $O.ks_tests.log 2>&1 || { echo tests failed; tail -30 $O.ks_tests.log; exit 1; }
grep -E "passed|failed" $O.ks_tests.log | tail -1
timeout -k 10 200 python -u tools/attn_bench.py --model-path --variant attn_fwd_ks=0,1 --rounds 3 > $O.ks_bench.log 2>&1 || { echo bench failed; tail $O.ks_bench.log; exit 1; }
tail -4 $O.ks_bench.log
