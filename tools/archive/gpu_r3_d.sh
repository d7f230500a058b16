#!/bin/bash
# Round 3: split-at-stash prefetch depth (FLR_PREFETCH=3: two tiles of global loads
# in flight) — bit-identity, then conv / batched-GEMM timing vs depth 2, same process.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_pf_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_PREFETCH=3" > gpurun_out/r3_conv_pf.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_PREFETCH=3" > gpurun_out/r3_bgemm_pf.txt 2>&1 || exit 1
