#!/bin/bash
# Round 3: PMC passes (separate runs, SQ counters only) over the C4 attention kernels.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/att_bench.py > gpurun_out/r3z_att_bench.txt 2>&1 || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_WAIT_INST_LDS"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc_att_$i -o p -- python3 tools/att_bench.py > gpurun_out/r3z_pmc_att_$i.log 2>&1 || exit 1
  python3 tools/pmc_stats.py /tmp/pmc_att_$i/p_results.db > gpurun_out/r3z_pmc_att_$i.txt 2>&1
done
cat gpurun_out/r3z_att_bench.txt
