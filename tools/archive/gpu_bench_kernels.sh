#!/bin/bash
# kernel microbenchmarks (in-process A/B variants)
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "${VARIANTS:-FLR_GEMM=A}" > gpurun_out/bgemm_bench.txt 2>&1
K=128 timeout -k 10 300 python -u tools/conv_bench.py --reps 5 --variants "${VARIANTS:-FLR_GEMM=A}" > gpurun_out/conv_bench.txt 2>&1
