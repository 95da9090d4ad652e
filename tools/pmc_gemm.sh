export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
for t in 0 4; do
  timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv --kernel-include-regex gemm -d gpurun_out/pmcg$t -o g -- python -u tools/gemm_bench.py one fwd.gate_up $t 5 > gpurun_out/pmcg$t.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv --kernel-include-regex gemm -d gpurun_out/pmch$t -o g -- python -u tools/gemm_bench.py one fwd.gate_up $t 5 > gpurun_out/pmch$t.log 2>&1 || exit 1
done
