#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pool_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/pool_bench.py > gpurun_out/pool_bench.txt 2>&1
