#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, separate passes) of the reference-exact kernels
set -o pipefail
mkdir -p gpurun_out/r5f
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export FLR_LIB=abl/xi0_cs64_abl0/libflr.so
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5f/fetch -o f --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5f/fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 gpurun_out/r5f/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r5f/hit -o h --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5f/hit.log 2>&1 || { echo "pmc hit failed"; tail -5 gpurun_out/r5f/hit.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d gpurun_out/r5f/sq -o s --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5f/sq.log 2>&1 || { echo "pmc sq failed"; tail -5 gpurun_out/r5f/sq.log; exit 1; }
echo done
