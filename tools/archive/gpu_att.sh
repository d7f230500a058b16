#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_xfmr.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/att_tests.log 2>&1
echo rc=$? >> gpurun_out/att_tests.log
timeout -k 10 120 python -u tools/att_bench.py > gpurun_out/att_bench.txt 2>&1
