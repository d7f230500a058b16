#!/bin/bash
# Round 3: the double-buffered split-at-stash GEMM (FLR_GEMM=db) — bit-identity
# tests, then conv / batched-GEMM timing against the default form, same process.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  -k "forms or addend" > gpurun_out/r3_db_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_GEMM=db" > gpurun_out/r3_conv_db.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_GEMM=db" > gpurun_out/r3_bgemm_db.txt 2>&1 || exit 1
