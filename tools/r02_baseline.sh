#!/bin/bash
# Round-2 baseline on a fresh box: GPU parity suite, bench, kernel trace, attention PMC at
# d64 S1024 (SmolLM) and d128 S4096 (Llama-2-7B CP=8 block), GEMM traffic at grad_acc 2.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02a}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/${T}_bench.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/${T}_pytest.log; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -u tools/attn_bench.py --reps 20 > gpurun_out/${T}_attn64.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn_bench.py --reps 10 --B 1 --S 4096 --H 32 --D 128 > gpurun_out/${T}_attn128.log 2>&1 || exit 1
cat gpurun_out/${T}_attn64.log gpurun_out/${T}_attn128.log
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for cfg in "64:--reps 5" "128:--reps 3 --B 1 --S 4096 --H 32 --D 128"; do
  d=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv --kernel-include-regex attn -d gpurun_out/${T}_pmca1_$d -o a -- python -u tools/attn_bench.py $args > gpurun_out/${T}_pmca1_$d.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv --kernel-include-regex attn -d gpurun_out/${T}_pmca2_$d -o a -- python -u tools/attn_bench.py $args > gpurun_out/${T}_pmca2_$d.log 2>&1 || exit 1
done
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc1 -o f -- python -u bench.py --steps 1 --warmup 0 --grad-acc 2 --cpu-tokens 0 --no-probe > gpurun_out/${T}_pmc1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc2 -o w -- python -u bench.py --steps 1 --warmup 0 --grad-acc 2 --cpu-tokens 0 --no-probe > gpurun_out/${T}_pmc2.log 2>&1 || exit 1
find gpurun_out -name "*.db" -delete
echo done
