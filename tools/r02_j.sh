#!/bin/bash
# transposed-weight dX A/B (microbench + in-situ bench), AdamW A/B, new tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02j}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or adamw or embedding_sort" > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 200 python -u tools/dgrad_bt.py > gpurun_out/${T}_dgrad_bt.log 2>&1 || { echo dgrad_bt failed; tail gpurun_out/${T}_dgrad_bt.log; exit 1; }
cat gpurun_out/${T}_dgrad_bt.log
timeout -k 10 120 python -u tools/adamw_bench.py --old tools/ab/libadamw_old.so > gpurun_out/${T}_adamw.log 2>&1 || { echo adamw failed; tail gpurun_out/${T}_adamw.log; exit 1; }
cat gpurun_out/${T}_adamw.log
for i in 1 2; do
  for f in 0 1; do
    PICOTRON_WT=$f timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_wt$f$i.json 2>/dev/null || { echo "bench $f failed"; exit 1; }
    echo "wt=$f: $(cut -c1-200 gpurun_out/${T}_wt$f$i.json)"
  done
done
