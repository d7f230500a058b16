#!/bin/bash
# where the rocprofv3 --kernel-trace crash in the K=256 C4 graph replay sits.
# One run: capture, dump /proc/self/maps, replay under the profiler; the crash's native frames are
# mapped onto the libraries afterwards (tools/symbolize_maps.py, on the CPU side).
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r4prof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pr -o b -- python3 -X faulthandler "$R/tools/replay_maps.py" bench "$R/gpurun_out/r4prof/c4_K256.maps" --config C4 --clients 256 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4prof/c4_K256_replay.log" 2>&1
echo "rc=$?"
grep -v "simple_timer\|SQLite3" "$R/gpurun_out/r4prof/c4_K256_replay.log" | head -50

cd "$R"
if grep -q '"metric"' gpurun_out/r4prof/c4_K256_replay.log; then
  python3 tools/rocpd_stats.py /tmp/pr/b_results.db > gpurun_out/r4prof/c4_K256_graph_kernel_stats.txt 2>&1
  head -14 gpurun_out/r4prof/c4_K256_graph_kernel_stats.txt | cut -c1-200
fi
