#!/bin/bash
# full GPU suite; TP / CP per-rank compute proxies; N-rank bench rehearsal over gloo on one GPU
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 3 > gpurun_out/${T}_tpproxy.json 2> gpurun_out/${T}_tpproxy.err || { echo tpproxy failed; tail gpurun_out/${T}_tpproxy.err; exit 1; }
cat gpurun_out/${T}_tpproxy.json
timeout -k 10 300 python -u bench.py --cp-proxy 8 --model llama2-7b --seq 32768 --mbs 1 --steps 3 > gpurun_out/${T}_cpproxy.json 2> gpurun_out/${T}_cpproxy.err || { echo cpproxy failed; tail gpurun_out/${T}_cpproxy.err; exit 1; }
cat gpurun_out/${T}_cpproxy.json
for cfg in "--tp 2" "--cp 2" "--tp 2 --dp-bucket"; do
  timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --backend gloo $cfg --layers 2 --grad-acc 2 --steps 1 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_rehearse.log 2>&1 || { echo "rehearsal $cfg failed"; tail -30 gpurun_out/${T}_rehearse.log; exit 1; }
  echo "rehearsal $cfg:"; tail -1 gpurun_out/${T}_rehearse.log | cut -c1-400
done
timeout -k 10 400 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_llama.json 2> gpurun_out/${T}_llama.err || { echo llama failed; tail gpurun_out/${T}_llama.err; exit 1; }
cut -c1-600 gpurun_out/${T}_llama.json
