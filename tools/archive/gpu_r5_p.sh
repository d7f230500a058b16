#!/bin/bash
# kernel summaries of a C3 round: reference-exact distances (torch order) vs Gram (training order)
set -o pipefail
mkdir -p gpurun_out/r5p
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in reference gram; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p/$m -o p -- python3 -u bench.py --steps 4 --warmup 1 --pairwise $m --no-cpu-baseline > gpurun_out/r5p/$m.log 2>&1 || { echo "prof $m failed"; tail -20 gpurun_out/r5p/$m.log; exit 1; }
  python3 tools/rocpd_stats.py gpurun_out/r5p/$m/p_results.db > gpurun_out/r5p/stats_$m.txt && head -30 gpurun_out/r5p/stats_$m.txt
done
