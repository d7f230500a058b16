#!/bin/bash
# Round 3: kernel summary of the C4/C5 aggregation kernels (K = 512 Gram breakdown).
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pa -o a -- python3 "$R/tools/agg_c4c5.py" > "$R/gpurun_out/r3s_prof.log" 2>&1 || exit 1
cd "$R" && python3 tools/rocpd_stats.py /tmp/pa/a_results.db > gpurun_out/r3s_agg_kernel_stats.txt
