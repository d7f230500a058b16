# PMC stall breakdown of the conv kernels: usage LAYERS="l1 l3b" bash tools/archive/pmc_conv.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LAYERS:-l1 l3b}; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA -d /tmp/pmc_$L -o p -- python3 tools/conv_bench.py --only $L --reps 2 > gpurun_out/pmc_$L.log 2>&1 || exit $?
  python3 tools/pmc_stats.py /tmp/pmc_$L/p_results.db > gpurun_out/pmc_$L.txt 2>&1
  cat gpurun_out/pmc_$L.txt
done
