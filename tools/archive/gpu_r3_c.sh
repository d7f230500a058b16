#!/bin/bash
# Round 3: the transposed-image weight gradient (wsgemm_kernel, default for WgtT) —
# bit-identity vs the per-wave-split form and norm partials, then conv + GEMM timing
# (default vs FLR_GEMM=pipe, same process) and the C3 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_ws_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_GEMM=pipe" > gpurun_out/r3_conv_ws.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bgemm_bench.py > gpurun_out/r3_bgemm.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_bench_c3_ws.json 2> gpurun_out/r3_bench_c3_ws.err || exit 1
