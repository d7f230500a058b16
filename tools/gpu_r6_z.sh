#!/bin/bash
# round 6: SQ counters of the 4-wave and 8-wave ping-pong batched GEMM at one shape
set -o pipefail
O=gpurun_out/r6z2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  FLR_GEMM_PP8=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS -d /tmp/pp$v -o p -- python3 tools/pp_one.py > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  python3 tools/pmc_stats.py $(ls /tmp/pp$v/*/p_results.db /tmp/pp$v/p_results.db 2>/dev/null | head -1) > $O/pmc_$v.txt 2>&1 || { echo "stats $v"; tail -5 $O/pmc_$v.txt; ls -R /tmp/pp$v | head; exit 1; }
  echo "== pp8=$v"; grep -E "gemm" $O/pmc_$v.txt | cut -c1-140 | head -20
done
