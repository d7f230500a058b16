#!/bin/bash
# PMC passes over the reference-exact distance kernels (one counter set per run)
set -o pipefail
mkdir -p gpurun_out/r5pmc2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 -d gpurun_out/r5pmc2/$1 -o p -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5pmc2/$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 gpurun_out/r5pmc2/$1.log; exit 1; }
  python3 tools/pmc_stats.py gpurun_out/r5pmc2/$1/p_results.db | grep -E "kernel  |pwref" > gpurun_out/r5pmc2/$1.txt && cat gpurun_out/r5pmc2/$1.txt
}
run a "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS" &&
run b "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" &&
run c "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU" &&
run d "FETCH_SIZE"
