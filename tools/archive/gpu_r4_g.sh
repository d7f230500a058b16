#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/diag_step0_fp64.py 32 0 3 > gpurun_out/r4g_step0_fp64.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4g_step0_fp64.txt | tail -14
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk16 -o b -- python3 "$R/bench.py" --clients 16 --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r4g_prof_k16.log" 2>&1 || { echo "prof rc=$?"; tail -5 "$R/gpurun_out/r4g_prof_k16.log"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pk16/b_results.db > gpurun_out/r4g_k16_kernel_stats.txt 2>&1
head -25 gpurun_out/r4g_k16_kernel_stats.txt | cut -c1-160
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4g_prof_k16.log
