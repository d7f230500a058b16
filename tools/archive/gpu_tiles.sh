#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/tiles_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/conv_bench.py --reps 40 > gpurun_out/tiles.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/round_ab.py > gpurun_out/round_ab.txt 2>&1
