#!/bin/bash
# C3 rocprofv3 kernel summary with the text branch on the caller's stream (FLR_TEXT_STREAM=0): per-kernel
# durations free of the text stream's concurrency, for the conv utilisation figure
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/final
export FLR_TEXT_STREAM=0
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pser -o b -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/final/prof_c3_serial.log" 2>&1 || { echo "prof rc=$?"; tail -10 "$R/gpurun_out/final/prof_c3_serial.log"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pser/b_results.db > gpurun_out/final/r4_c3_kernel_stats_serial.txt 2>&1
head -8 gpurun_out/final/r4_c3_kernel_stats_serial.txt | cut -c1-150
unset FLR_TEXT_STREAM
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pk16b -o b -- python3 "$R/bench.py" --clients 16 --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/final/prof_k16.log" 2>&1 || { echo "prof k16 rc=$?"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pk16b/b_results.db > gpurun_out/final/r4_k16_kernel_stats.txt 2>&1
head -30 gpurun_out/final/r4_k16_kernel_stats.txt | cut -c1-150
