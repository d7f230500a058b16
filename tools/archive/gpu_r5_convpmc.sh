#!/bin/bash
# SQ counters of every kernel of a C3 round (one pass, 8 SQ counters) — the conv /
# GEMM main loop's MFMA busy share and waits, for the next round's work
set -o pipefail
D=gpurun_out/r5convpmc; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $D/pmc -o p -- python3 -u bench.py --no-cpu-baseline --steps 1 --warmup 0 > $D/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $D/pmc.log; exit 1; }
python3 tools/pmc_stats.py $D/pmc/p_results.db > $D/pmc.txt && rm -rf $D/pmc && grep -c . $D/pmc.txt
