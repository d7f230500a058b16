#!/bin/bash
# Round 4: the rocprofv3 --kernel-trace crash inside the replay of the C4 round graph.
# Graph node counts first, then rocprofv3 --kernel-trace --stats on C4 rounds with the graph ON at
# growing K; the first failing K ends the call (its log is kept), a clean K=256 gives the C4 summary.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r4prof
for K in 64 256; do
  timeout -k 10 300 python -u tools/graph_nodes.py C4 $K >> gpurun_out/r4prof/graph_nodes.txt 2>&1 || { echo "graph_nodes K=$K rc=$?"; exit 1; }
done
cat gpurun_out/r4prof/graph_nodes.txt
for K in 64 128 256; do
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pc4_$K -o b -- python3 -X faulthandler "$R/bench.py" --config C4 --clients $K --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4prof/c4_K${K}.log" 2>&1
  rc=$?
  cd "$R"
  echo "C4 K=$K graph-replayed under rocprofv3: rc=$rc"
  tail -25 gpurun_out/r4prof/c4_K${K}.log
  if [ $rc -ne 0 ]; then exit 0; fi
  python3 tools/rocpd_stats.py /tmp/pc4_$K/b_results.db > gpurun_out/r4prof/c4_K${K}_kernel_stats.txt 2>&1 || true
  head -5 gpurun_out/r4prof/c4_K${K}_kernel_stats.txt
done
