#!/bin/bash
# Round 3 (current code): C4 and C5 bench lines and the C4 rocprofv3 kernel summary (eager launches, FLR_GRAPH=0:
# rocprofv3 --kernel-trace segfaulted inside the replay of the K = 256 round graph).
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
# (C4 line: the previous call)

cd /tmp && FLR_GRAPH=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/pc4 -o b -- python3 "$R/bench.py" --config C4 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/c45_prof_c4.log" 2>&1 || exit 1
cd "$R" && python3 tools/rocpd_stats.py /tmp/pc4/b_results.db > gpurun_out/c45_c4_kernel_stats.txt || exit 1
timeout -k 10 600 python -u bench.py --config C5 --steps 2 --warmup 1 > gpurun_out/c45_bench_c5.json 2> gpurun_out/c45_bench_c5.err || exit 1
tail -1 gpurun_out/c45_bench_c5.json | cut -c1-200
