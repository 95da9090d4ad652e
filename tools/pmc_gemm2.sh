#!/bin/bash
# PMC passes (one counter set per run) over single-shape GEMM launches (tools/gemm_bench.py one)
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02g}
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
C3="SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_COUNT"
for job in "fwd.gate_up 12" "dgrad.gate_up 13" "fwd.o 13" "wgrad.gate_up 12" "swiglu_bwd 0" "fwd.down 13"; do
  set -- $job
  n=${1//./_}_$2
  timeout -k 10 120 python -u tools/gemm_bench.py one $1 $2 10 > gpurun_out/${T}_${n}.time 2>&1 || exit 1
  for i in 1 2 3; do
    eval C=\$C$i
    timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv --kernel-include-regex gemm -d gpurun_out/${T}_${n}_p$i -o g -- python -u tools/gemm_bench.py one $1 $2 5 > gpurun_out/${T}_${n}_p$i.log 2>&1 || { echo "pmc $n $i failed"; tail -3 gpurun_out/${T}_${n}_p$i.log; exit 1; }
  done
  cat gpurun_out/${T}_${n}.time
done
find gpurun_out -name "*.db" -delete
