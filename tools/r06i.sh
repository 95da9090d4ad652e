set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -k "g8 or g11" -m gpu -x -q --timeout 300 --timeout-method thread > $O.pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error|assert" $O.pytest.log | head -20; exit 1; }
tail -1 $O.pytest.log
timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 5 > $O.tp.json 2> $O.tp.err || { echo tp failed; tail -5 $O.tp.err; exit 1; }
python -c "import json; d=json.load(open('$O.tp.json')); print('tp8 proxy', round(d['value']), round(d['ms_per_microbatch'],2), round(d['eager_ms_per_microbatch'],2), d['launch'])"
