#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_bench.py --only stem --reps 10 --variants "FLR_STEM=gather;FLR_STEM=col" > gpurun_out/stem_bench.txt 2>&1
