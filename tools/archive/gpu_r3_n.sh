#!/bin/bash
# Round 3: C3 bench line + its rocprofv3 kernel summary (same command).
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u bench.py > gpurun_out/r3n_bench_c3.json 2> gpurun_out/r3n_bench_c3.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r3n_prof_c3.log" 2>&1 || exit 1
cd "$R" && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/r3n_c3_kernel_stats.txt
