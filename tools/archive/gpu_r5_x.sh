#!/bin/bash
# round-5 bench lines on the final library: C2, C4, C5 (each with its cpu_baseline), and
# the rocprofv3 kernel summary of the default C3 command
set -o pipefail
mkdir -p gpurun_out/r5x
for c in C2 C4 C5; do
  timeout -k 10 420 python -u bench.py --config $c > gpurun_out/r5x/bench_$c.json 2> gpurun_out/r5x/bench_$c.err || { echo "bench $c failed"; tail -20 gpurun_out/r5x/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r5x/bench_$c.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['aggregate_ms'], d.get('aggregate_ms_by_defense'), (d.get('distance_phase') or {}).get('ms'))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5x/prof -o p -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5x/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5x/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5x/prof/p_results.db > gpurun_out/r5x/c3_stats.txt && head -8 gpurun_out/r5x/c3_stats.txt
