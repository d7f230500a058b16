#!/bin/bash
set -u
cd "$(dirname "$0")/.."
for v in 8 16 32; do
  FLR_CONV_MINKT=$v timeout -k 10 200 python -u tools/conv_bench.py --reps 10 > gpurun_out/minkt_$v.txt 2>&1 || exit 1
done
