#!/bin/bash
# C4 (K=256) rocprofv3 kernel summary with the round graph replayed.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r4prof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pc4 -o b -- python3 -X faulthandler "$R/bench.py" --config C4 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4prof/c4_K256_graph.log" 2>&1
rc=$?
echo "rc=$rc"
cd "$R"
grep -v "simple_timer\|SQLite3" gpurun_out/r4prof/c4_K256_graph.log | tail -30 | cut -c1-300
[ $rc -eq 0 ] || exit 0
python3 tools/rocpd_stats.py /tmp/pc4/b_results.db > gpurun_out/r4prof/c4_K256_graph_kernel_stats.txt 2>&1
head -12 gpurun_out/r4prof/c4_K256_graph_kernel_stats.txt | cut -c1-200
