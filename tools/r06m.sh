set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py -k "tp8 or tensor_parallel_llama_tp2" > $O.tp_tests.log 2>&1 || { echo tests failed; tail -30 $O.tp_tests.log; exit 1; }
tail -3 $O.tp_tests.log
GRID8="tp8mb32|--tp 8 --layers 2 --mbs 32 --grad-acc 1" bash tools/gpu.sh $1 grid8
