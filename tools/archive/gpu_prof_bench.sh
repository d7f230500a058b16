#!/bin/bash
# rocprofv3 kernel summary of a short C3 bench -> gpurun_out/prof_bench_stats.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > /root/repo/gpurun_out/prof_bench.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_bench_stats.txt
