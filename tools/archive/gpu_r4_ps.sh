#!/bin/bash
# pre-split batched GEMM: bit-identity vs split-at-stash, timing A/B at the encoder shapes, C4 bench
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bgemm_dma.py tests/test_gpu_bgemm.py tests/test_gpu_conv.py -k "bgemm or presplit" > gpurun_out/r4ps_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4ps_tests.log; exit 1; }
tail -1 gpurun_out/r4ps_tests.log
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_BGEMM_PRESPLIT=0" > gpurun_out/r4ps_bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r4ps_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4ps_bench.txt
