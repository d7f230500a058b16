#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py tests/test_gpu_xfmr.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --reps 10 --variants "${VARIANTS:-FLR_GEMM=old}" > gpurun_out/conv_bench.txt 2>&1
