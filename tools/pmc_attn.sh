# PMC passes over tools/attn_bench.py (one counter set per run; see MI355X_MICROARCH.md PMC limits)
export TMPDIR=/tmp
mkdir -p gpurun_out
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv --kernel-include-regex attn -d gpurun_out/pmca1 -o a -- python -u tools/attn_bench.py --reps 5 > gpurun_out/pmca1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv --kernel-include-regex attn -d gpurun_out/pmca2 -o a -- python -u tools/attn_bench.py --reps 5 > gpurun_out/pmca2.log 2>&1 || exit 1
find gpurun_out -name "*.db" -delete
