#!/bin/bash
# full GPU suite; default bench line; its kernel-trace profile; TP proxy; 1-GPU DP bucket hook overhead
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 3 > gpurun_out/${T}_tpproxy.json 2> gpurun_out/${T}_tpproxy.err || { echo tpproxy failed; tail gpurun_out/${T}_tpproxy.err; exit 1; }
cat gpurun_out/${T}_tpproxy.json
for cfg in "--bucket-mb 25 --grad-type fp32" "--bucket-mb 100 --grad-type fp32" "--bucket-mb 400 --grad-type fp32" "--bucket-mb 25 --grad-type bf16" "--bucket-mb 100 --grad-type bf16"; do
  timeout -k 10 300 python -u bench.py --dp-bucket $cfg --grad-acc 8 --steps 3 --cpu-tokens 0 > gpurun_out/${T}_dp.json 2> gpurun_out/${T}_dp.err || { echo "dp $cfg failed"; tail gpurun_out/${T}_dp.err; exit 1; }
  echo "dp $cfg: $(cut -c1-300 gpurun_out/${T}_dp.json)" | tee -a gpurun_out/${T}_dpstudy.log
done
timeout -k 10 300 python -u bench.py --grad-acc 8 --steps 3 --cpu-tokens 0 > gpurun_out/${T}_nodp.json 2>&1 && echo "no dp wrapper: $(cut -c1-300 gpurun_out/${T}_nodp.json)" | tee -a gpurun_out/${T}_dpstudy.log
