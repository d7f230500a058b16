export TMPDIR=/tmp
timeout -k 10 120 python tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 || exit $?
cat gpurun_out/conv_bench.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
for L in l1 l2b; do
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA -d /tmp/pmc_$L -o p -- python3 tools/conv_bench.py --only $L --reps 2 > gpurun_out/pmc_$L.log 2>&1 || exit $?
  python3 tools/pmc_stats.py /tmp/pmc_$L/p_results.db > gpurun_out/pmc_$L.txt 2>&1
done
