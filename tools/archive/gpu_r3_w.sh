#!/bin/bash
# Round 3: producer / consumer split-at-stash kernel (FLR_SG_PC=1) — conv / GEMM bit-identity under it,
# per-layer and per-shape timing against the one-stage kernel (same process), C3 bench both ways.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FLR_SG_PC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bgemm.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_SG_PC=1" > gpurun_out/r3w_conv.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_SG_PC=1" > gpurun_out/r3w_bgemm.txt 2>&1 || exit 1
for v in 0 1 0 1; do
  FLR_SG_PC=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3w_bench_$v.json 2>/dev/null || exit 1
done
