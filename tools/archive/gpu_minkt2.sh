#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py tests/test_gpu_shard.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/minkt_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/round_ab.py > gpurun_out/round_ab_32.txt 2>&1 || exit 1
FLR_CONV_MINKT=8 timeout -k 10 200 python -u tools/round_ab.py > gpurun_out/round_ab_8.txt 2>&1
