#!/bin/bash
# Round 3: GRU "8,2s" with non-temporal streamed-once operands — bit-identity and timing.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gru_bench.py > gpurun_out/r3u_gru.txt 2>&1 || exit 1
