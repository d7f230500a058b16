#!/bin/bash
# Round 3: (1) double-buffered split-at-stash kernel (FLR_SG_DB=2|3) — conv / GEMM
# bit-identity under it, per-layer timing vs the single-stage kernel (same process);
# (2) the side-stream optimizer overlap — tests, C3 bench on / off.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FLR_SG_DB=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bgemm.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3j_db_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_SG_DB=2;FLR_SG_DB=3" > gpurun_out/r3j_conv.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_SG_DB=2;FLR_SG_DB=3" > gpurun_out/r3j_bgemm.txt 2>&1 || exit 1
bash tools/archive/gpu_r3_i.sh
