#!/bin/bash
# Round 3: fused stem BN + ReLU + max-pool — tests, C3 bench + kernel summary.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_pool.py tests/test_gpu_native_trainer.py \
  tests/test_gpu_round.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || exit 1
bash tools/archive/gpu_r3_n.sh
