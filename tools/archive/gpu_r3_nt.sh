#!/bin/bash
# Round 3: dead-range copy with plain vs non-temporal stores (FLR_DEAD_NT), kernel time per C3 round.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
for v in 0 1 0 1; do
  cd /tmp && FLR_SGD_NT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/snt$v -o b -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/nt_prof_$v.log" 2>&1 || exit 1
  cd "$R" && python3 tools/rocpd_stats.py /tmp/snt$v/b_results.db > gpurun_out/nt_stats_$v.txt
  echo "variant $v"; head -1 gpurun_out/nt_stats_$v.txt; grep -E "dead_ranges|sgd_blocked|gram_partials" gpurun_out/nt_stats_$v.txt | cut -c1-40,90-140
done
