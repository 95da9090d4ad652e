#!/bin/bash
# lm_head CE statistics: tests, then bench A/B (PICOTRON_CE_STATS=1/0 interleaved), kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02f}
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" gpurun_out/${T}_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  for f in 1 0; do
    PICOTRON_CE_STATS=$f timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 > gpurun_out/${T}_b$f$i.json 2>/dev/null || { echo "bench $f failed"; exit 1; }
    echo "stats=$f: $(cut -c1-200 gpurun_out/${T}_b$f$i.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python -u bench.py --steps 1 --warmup 1 --cpu-tokens 0 > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
grep -E "Li8EE|ce_fwd|Li0EE" gpurun_out/${T}_prof/${T}_kernel_stats.csv | cut -c1-200
