#!/bin/bash
# Round 3: far-cluster refine + sharded phases + the trained-C3 Krum record, then
# the conv tile sweep (FLR_CONV_TILE variants, same process).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "pairwise or shard or c3_trained" > gpurun_out/r3_t2.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/conv_bench.py --variants "FLR_CONV_TILE=14;FLR_CONV_TILE=41;FLR_CONV_TILE=13;FLR_CONV_TILE=31;FLR_CONV_TILE=22;FLR_CONV_TILE=12;FLR_CONV_TILE=21;FLR_CONV_TILE=11" > gpurun_out/r3_conv_tiles.txt 2>&1 || exit 1
