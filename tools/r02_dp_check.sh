#!/bin/bash
# DP path end to end: the real-shape f32 main_grad layer test, a 2-rank DataParallelBucket bench over
# gloo on one GPU (timing meaningless) and the 1-rank RCCL --dp-bucket bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02dp}
timeout -k 10 300 python -u -m pytest tests/test_shapes_gpu.py tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 --grad-acc 4 --cpu-tokens 0 > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { echo gloo2 failed; tail -20 gpurun_out/${T}_gloo2.err; exit 1; }
cut -c1-300 gpurun_out/${T}_gloo2.json
for gt in fp32 bf16; do
  timeout -k 10 300 python -u bench.py --dp-bucket --grad-type $gt --steps 3 --cpu-tokens 0 > gpurun_out/${T}_dp_$gt.json 2>/dev/null || { echo dp $gt failed; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_dp_$gt.json')); print('dp-bucket $gt', round(d['value']), round(d['ms_per_step'],1))"
done
timeout -k 10 300 python -u bench.py --steps 3 --cpu-tokens 0 > gpurun_out/${T}_plain.json 2>/dev/null || { echo plain failed; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_plain.json')); print('plain', round(d['value']), round(d['ms_per_step'],1))"
