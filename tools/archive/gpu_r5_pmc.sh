#!/bin/bash
# PMC pass over the reference-exact distance kernels (one counter set per run)
set -o pipefail
mkdir -p gpurun_out/r5pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d gpurun_out/r5pmc/a -o a --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5pmc/a.log 2>&1 || { echo "pmc a failed"; tail -5 gpurun_out/r5pmc/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/r5pmc/b -o b --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5pmc/b.log 2>&1 || { echo "pmc b failed"; tail -5 gpurun_out/r5pmc/b.log; exit 1; }
find gpurun_out/r5pmc -name "*counter_collection.csv" | head
