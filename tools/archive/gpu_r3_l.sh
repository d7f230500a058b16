#!/bin/bash
# Round 3: side-stream optimizer priority A/B (C3 bench, same box): off / normal / low / high.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  FLR_SGD_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3l_off.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3l_normal.json 2>/dev/null || exit 1
  FLR_SGD_PRIO=low timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3l_low.json 2>/dev/null || exit 1
  FLR_SGD_PRIO=high timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3l_high.json 2>/dev/null || exit 1
done
