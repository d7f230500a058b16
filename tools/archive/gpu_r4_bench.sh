#!/bin/bash
# Round 4 bench lines for C2 / C4 / C5 (and C3) with the per-aggregator cpu_baseline.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for C in ${CONFIGS:-C2 C4 C5}; do
  case $C in C2|C3) S=10;; *) S=3;; esac
  timeout -k 10 500 python3 -u bench.py --config $C --steps $S --warmup 1 > gpurun_out/r4_bench_$C.log 2>&1 || { echo "bench $C rc=$?"; tail -20 gpurun_out/r4_bench_$C.log; exit 1; }
  grep '^{"metric' gpurun_out/r4_bench_$C.log > gpurun_out/r4_bench_$C.json
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r4_bench_$C.json')); c=d['cpu_baseline']; print('$C', d['value'], d['ms_per_step'], d.get('aggregate_ms_by_defense'), c['value'], c['aggregate_ms'], c['local_update_s_per_client'])"
done
