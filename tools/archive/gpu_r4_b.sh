#!/bin/bash
# round 4: the whole GPU suite (records -> gpurun_out/records), then the C3 bench under rocprofv3 --stats
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export FLR_RECORD_DIR=$R/gpurun_out/records
timeout -k 10 1500 python -u -m pytest -v -m gpu --timeout 900 --timeout-method thread tests > gpurun_out/r4b_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4b_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r4b_gpu_tests.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pc3 -o b -- python3 "$R/bench.py" --steps 8 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4b_prof_c3.log" 2>&1 || { echo "prof rc=$?"; tail -20 "$R/gpurun_out/r4b_prof_c3.log"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pc3/b_results.db > gpurun_out/r4b_c3_kernel_stats.txt 2>&1
head -30 gpurun_out/r4b_c3_kernel_stats.txt | cut -c1-150
grep -E "refine|gram|rows_mean|ref_norm" gpurun_out/r4b_c3_kernel_stats.txt | cut -c1-150
