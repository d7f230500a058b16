#!/bin/bash
# Round 3: where the fused GRU step's W_hh stream comes from: PMC passes (separate runs)
# FETCH_SIZE (L2 -> fabric: MALL or HBM) and TCC_HIT / TCC_MISS over tools/gru_bench.py.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for P in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/gpmc_$i -o p -- python3 tools/gru_bench.py > gpurun_out/gru_pmc_$i.log 2>&1 || exit 1
  python3 tools/pmc_stats.py /tmp/gpmc_$i/p_results.db | grep -E "fused|counter" > gpurun_out/gru_pmc_$i.txt 2>&1
  cat gpurun_out/gru_pmc_$i.txt | cut -c1-60,70-140
done
