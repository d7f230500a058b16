#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py tests/test_gpu_xfmr.py tests/test_gpu_gru.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/stash_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/round_ab.py FLR_GEMM=pipe FLR_GEMM=old > gpurun_out/round_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/stash_bench.json 2> gpurun_out/stash_bench.err
