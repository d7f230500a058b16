#!/bin/bash
# dot2 split: bit check, conv/train tests, per-layer conv timings.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hip/split_check > gpurun_out/split_check.txt 2>&1; cat gpurun_out/split_check.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py tests/test_gpu_bgemm.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench_dot2.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/split_bench.json 2> gpurun_out/split_bench.err || exit 1
tail -1 gpurun_out/split_bench.json | cut -c1-200
