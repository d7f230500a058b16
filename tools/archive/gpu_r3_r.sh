#!/bin/bash
# Round 3: K > 128 Gram cross groups 4 x 4 (NL = 8) — pairwise / Krum / shard tests, then the
# C4 / C5 aggregation timings against the 2 x 4 groups (abl/ni2), same box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_shard.py tests/test_gpu_krum_c3.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/r3r_agg_main.txt 2>&1 || exit 1
FLR_LIB=$PWD/abl/ni2/libflr.so timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/r3r_agg_ni2.txt 2>&1 || exit 1
