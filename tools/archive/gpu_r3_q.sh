#!/bin/bash
# Round 3: C2 / C4 / C5 bench lines (with the CPU baseline) and the C4 / C5 aggregation kernels.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config C2 > gpurun_out/r3q_bench_c2.json 2> gpurun_out/r3q_bench_c2.err || exit 1
timeout -k 10 500 python -u bench.py --config C4 --steps 2 --warmup 1 \
  --kernel-stats profiles/r3_c4_kernel_stats.txt > gpurun_out/r3q_bench_c4.json 2> gpurun_out/r3q_bench_c4.err || exit 1
timeout -k 10 600 python -u bench.py --config C5 --steps 2 --warmup 1 > gpurun_out/r3q_bench_c5.json 2> gpurun_out/r3q_bench_c5.err || exit 1
timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/r3q_agg_c4c5.txt 2>&1 || exit 1
