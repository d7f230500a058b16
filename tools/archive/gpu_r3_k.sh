#!/bin/bash
# Round 3: kernel trace of the C3 bench with the side-stream optimizer overlap on /
# off: how much of the optimizer's time runs concurrently with other kernels.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
for v in 1 0; do
  cd /tmp && FLR_SGD_OVERLAP=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ov$v -o t -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r3k_prof_$v.log" 2>&1 || exit 1
  cd "$R" && python3 tools/overlap_stats.py /tmp/ov$v/t_results.db sgd_blocked > gpurun_out/r3k_overlap_$v.txt 2>&1
  python3 tools/overlap_stats.py /tmp/ov$v/t_results.db sgd_blocked --after-last gram_partials >> gpurun_out/r3k_overlap_$v.txt 2>&1
done
