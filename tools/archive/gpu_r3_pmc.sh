#!/bin/bash
# PMC passes (separate runs, SQ counters only) over conv layers l1 / l3b and the ViT qkv GEMM.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL"
for L in l1 l3b; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc_${L}_$i -o p -- python3 tools/conv_bench.py --only $L --reps 2 > gpurun_out/r3_pmc_${L}_$i.log 2>&1 || exit 1
    python3 tools/pmc_stats.py /tmp/pmc_${L}_$i/p_results.db > gpurun_out/r3_pmc_${L}_$i.txt 2>&1
  done
done
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  ONLY=vit.qkv timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc_qkv_$i -o p -- python3 tools/bgemm_bench.py > gpurun_out/r3_pmc_qkv_$i.log 2>&1 || exit 1
  python3 tools/pmc_stats.py /tmp/pmc_qkv_$i/p_results.db > gpurun_out/r3_pmc_qkv_$i.txt 2>&1
done
