#!/bin/bash
# LDS-DMA batched GEMM: bit-identity vs the split-at-stash form, then timing A/B at the encoder shapes.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bgemm_dma.py tests/test_gpu_bgemm.py > gpurun_out/r4_dma_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_dma_tests.log; exit 1; }
tail -2 gpurun_out/r4_dma_tests.log
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_BGEMM_DMA=0" > gpurun_out/r4_dma_bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r4_dma_bench.txt; exit 1; }
cat gpurun_out/r4_dma_bench.txt
