#!/bin/bash
# End-of-session evidence on the final tree: GPU parity suite, smoke, bench (2 runs), rocprofv3
# kernel trace + stats of the bench, GEMM HBM traffic from separate FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02s3}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || { echo bench failed; tail gpurun_out/${T}_bench$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench$i.json')); print('bench', round(d['value']), round(d['ms_per_step'],1), round(d['mfu'],4), round(d['roofline']['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o k -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
gzip -f gpurun_out/${T}_prof/k_kernel_trace.csv
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc1 -o f -- python -u bench.py --steps 1 --warmup 0 --grad-acc 2 --cpu-tokens 0 --no-probe > gpurun_out/${T}_pmc1.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc2 -o w -- python -u bench.py --steps 1 --warmup 0 --grad-acc 2 --cpu-tokens 0 --no-probe > gpurun_out/${T}_pmc2.log 2>&1 || { echo pmc2 failed; exit 1; }
python tools/traffic_summary.py gpurun_out/${T}_pmc1/f_counter_collection.csv gpurun_out/${T}_pmc2/w_counter_collection.csv gpurun_out/${T}_gemm_traffic.json
find gpurun_out -name "*.db" -delete
echo done
