# Two PMC passes over one conv layer (default vs FLR_GEMM=pipe in one process)
export TMPDIR=/tmp
mkdir -p gpurun_out
L=${LAYER:-l3b}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc2_$i -o p -- python3 tools/conv_bench.py --only $L --reps 2 --variants "FLR_GEMM=pipe" > gpurun_out/pmc2_$i.log 2>&1 || exit $?
  python3 tools/pmc_stats.py /tmp/pmc2_$i/p_results.db > gpurun_out/pmc2_${L}_$i.txt 2>&1
done
