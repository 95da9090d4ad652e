#!/bin/bash
# side-stream dX / SwiGLU-bwd beside dW (PICOTRON_STREAMS=1) vs serial: layer tests with streams on, bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02s}
PICOTRON_STREAMS=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2 3; do
  for f in 0 1; do
    PICOTRON_STREAMS=$f timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 --no-probe > gpurun_out/${T}_s$f$i.json 2>/dev/null || { echo "bench $f failed"; exit 1; }
    echo "streams=$f: $(cut -c90-200 gpurun_out/${T}_s$f$i.json)"
  done
done
