#!/bin/bash
# Round 3: diagonal refine pairs staged once; side-stream overlap test case — tests, C3 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_krum_c3.py tests/test_gpu_native_trainer.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3m_bench.json 2> gpurun_out/r3m_bench.err || exit 1
