#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/gru_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gru_bench.py > gpurun_out/gru_bench.txt 2>&1
