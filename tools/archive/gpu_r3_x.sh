#!/bin/bash
# Round 3: narrow-N conv tiles (l4) — conv tests incl. narrow vs 64-wide bit-identity, native trainer,
# per-layer timing against FLR_CONV_NARROW=0, C3 bench both ways.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_native_trainer.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_CONV_NARROW=0" > gpurun_out/r3x_conv.txt 2>&1 || exit 1
for v in 1 0 1 0; do
  FLR_CONV_NARROW=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3x_bench_$v.json 2>/dev/null || exit 1
done
