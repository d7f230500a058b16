#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for KK in 32 64; do
  timeout -k 10 300 python3 -u bench.py --clients $KK --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4_k$KK.log 2>&1 || { echo "k$KK rc=$?"; exit 1; }
  echo "C3 K=$KK $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_k$KK.log)"
done
timeout -k 10 500 python3 -u bench.py --config C2 --steps 10 --warmup 1 > gpurun_out/r4_bench_C2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
grep '^{"metric' gpurun_out/r4_bench_C2.log > gpurun_out/r4_bench_C2.json
grep -o '"value": [0-9.]*, "unit": "rounds/s", "n_gpus": 1, "steps": 10, "warmup": 1, "ms_per_step": [0-9.]*' gpurun_out/r4_bench_C2.json
