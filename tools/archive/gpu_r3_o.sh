#!/bin/bash
# Round 3: refine (packed fp32, prefetch) + in-place shortcut dgrad — tests, C3 bench + kernel summary.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_aggregation.py tests/test_gpu_krum_c3.py \
  tests/test_gpu_native_trainer.py tests/test_gpu_round.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3o_tests.log 2>&1 || exit 1
bash tools/archive/gpu_r3_n.sh
